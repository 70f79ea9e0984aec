"""Host GPU inventory without amdsmi: the shim's sysfs discovery (render nodes, PCI BDF order) and the
xGMI adjacency read from the KFD topology's io_links (type 11), on fake /sys trees
(``dstack_amd.server.testing.fake_amd_sysfs``)."""

import json
import os
import subprocess

import pytest

from dstack_amd.native_bin import shim_path
from dstack_amd.server.testing import fake_amd_sysfs

pytestmark = pytest.mark.skipif(not shim_path(), reason="native agents not built")


def _host_info(root):
    r = subprocess.run([shim_path(), "--host-info"], env=dict(os.environ, DSTACK_SYSFS_ROOT=str(root)),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_eight_gpu_board_fully_connected(tmp_path):
    h = _host_info(fake_amd_sysfs(tmp_path, 8))
    assert h["gpu_count"] == 8 and h["gpu_name"] == "MI355X" and h["gpu_memory"] == 288 * 1024
    xg = h["topology"]["xgmi"]
    assert len(xg) == 8 and all(xg[i][j] == (0 if i == j else 1) for i in range(8) for j in range(8))
    bdfs = [g["bdf"] for g in h["topology"]["gpus"]]
    assert bdfs == sorted(bdfs)


def test_missing_links_and_pcie_only(tmp_path):
    root = fake_amd_sysfs(tmp_path / "a", 4)
    # cut the 0<->3 link both ways: KFD node ids are GPU index + 1
    nodes = tmp_path / "a" / "sys" / "class" / "kfd" / "kfd" / "topology" / "nodes"
    for a, b in ((1, 4), (4, 1)):
        for ld in (nodes / str(a) / "io_links").iterdir():
            if f"node_to {b}\n" in (ld / "properties").read_text():
                (ld / "properties").write_text(f"type 2\nnode_from {a}\nnode_to {b}\nweight 40\n")
    xg = _host_info(root)["topology"]["xgmi"]
    assert xg[0][3] == 0 and xg[3][0] == 0 and xg[0][1] == 1 and xg[2][3] == 1
    xg = _host_info(fake_amd_sysfs(tmp_path / "b", 2, xgmi=False))["topology"]["xgmi"]
    assert xg == [[0, 0], [0, 0]]
