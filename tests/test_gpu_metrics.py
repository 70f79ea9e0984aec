"""amdsmi metrics on the real GPU through the native collector (`dstack-shim --gpu-metrics`, the
same code the runner samples every 10 s): VRAM, power, temperature, HBM controller activity and
the xGMI link state / traffic counters of an MI355X."""

import json
import subprocess

import pytest

from dstack_amd.native_bin import shim_path

pytestmark = pytest.mark.gpu


def test_native_gpu_metrics_on_mi355x():
    shim = shim_path()
    if not shim:
        pytest.fail("dstack-shim not built")
    out = subprocess.run([shim, "--gpu-metrics"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    gpus = json.loads(out.stdout.strip().splitlines()[-1])
    print(json.dumps(gpus))
    assert gpus, "amdsmi reported no GPU"
    g = gpus[0]
    assert g["gpu_memory_total_bytes"] > 250 * 2**30  # 288 GB HBM3E
    assert 0 < g["gpu_power_watts"] < 1500 and 0 < g["gpu_temperature_c"] < 120
    assert 0 <= g["gpu_util_percent"] <= 100
    x = g.get("xgmi")
    if x is not None:  # an OAM MI355X in an 8-GPU baseboard has 7 xGMI links
        assert 0 <= x["links_up"] <= x["links_total"] <= 8
        assert x["read_kb"] >= 0 and x["write_kb"] >= 0
