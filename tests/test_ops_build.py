"""The HIP extension build is content-addressed (ops/build.py): the digests change with any source,
header or flag, and a built tree reports itself current."""

import pytest

from dstack_amd.ops import build


def test_digest_tracks_content_and_flags(tmp_path):
    a = tmp_path / "k.hip"
    a.write_text("__global__ void k() {}\n")
    d1 = build._digest([a], ["hipcc", "-O3"])
    assert d1 == build._digest([a], ["hipcc", "-O3"])
    assert d1 != build._digest([a], ["hipcc", "-O2"])
    a.write_text("__global__ void k() { }\n")
    assert d1 != build._digest([a], ["hipcc", "-O3"])
    obj = tmp_path / "k.o"
    assert build._stale(obj, d1)
    obj.write_bytes(b"x")
    build._stamp(obj, d1)
    assert not build._stale(obj, d1) and build._stale(obj, d1 + "0")


def test_failed_build_leaves_no_stale_stamp(tmp_path, monkeypatch):
    """When one unit fails to compile, a unit that compiled in the same call carries the stamp of its
    NEW sources (or none) -- never the stamp of the previous ones, under which a revert of those
    sources would reuse the new object."""
    a_obj, b_obj = tmp_path / "a.o", tmp_path / "b.o"
    a_obj.write_bytes(b"old a")
    b_obj.write_bytes(b"old b")
    build._stamp(a_obj, "old-a")
    build._stamp(b_obj, "old-b")
    units = [(a_obj, ["cc", "a"], "new-a"), (b_obj, ["cc", "b"], "new-b")]

    def run(cmd):
        if cmd[1] == "b":
            raise RuntimeError("compile failed: b")
        a_obj.write_bytes(b"new a")
        return ""

    monkeypatch.setattr(build, "_quick_current", lambda: False)
    monkeypatch.setattr(build, "_plan", lambda keep_asm=False: (units, ["ld"], "so"))
    monkeypatch.setattr(build, "_run", run)
    monkeypatch.setattr(build, "check_toolchain", lambda: "hipcc")
    monkeypatch.setattr(build, "BUILD", tmp_path)
    with pytest.raises(RuntimeError, match="compile failed: b"):
        build.build()
    assert not build._stale(a_obj, "new-a")  # compiled: stamped with its new digest
    assert build._stale(a_obj, "old-a")
    assert build._stale(b_obj, "old-b") and build._stale(b_obj, "new-b")  # failed: no stamp at all


def test_plan_covers_every_kernel_source():
    units, link, digest = build._plan()
    srcs = {p.stem for p in build.CSRC.glob("*.hip")} | {"bindings"}
    assert {u[0].stem for u in units} == srcs
    assert any("--offload-arch=gfx950" in c for c in units[0][1]) and len(digest) == 64


def test_built_extension_is_current():
    if not build.so_path().exists():
        pytest.skip("extension not built in this checkout")
    assert build.is_current(), "the .so does not match the current kernel sources: rebuild"


def test_manifest_records_provenance_and_detects_foreign_binaries(tmp_path, monkeypatch):
    """The manifest next to the .so ties the binary to the kernel sources of this tree; a binary
    that is not the one the manifest describes, or a manifest for other sources, is refused."""
    import json
    import shutil

    if not build.so_path().exists() or not build.manifest_path().exists():
        pytest.skip("extension not built in this checkout")
    m = build.verify_loaded(str(build.so_path()))
    assert m["arch"] == "gfx950" and set(m["units"]) >= {"flash_attn", "elementwise", "bindings"}
    fake = tmp_path / "_C.so"
    shutil.copy(build.so_path(), fake)
    with open(fake, "ab") as f:
        f.write(b"\0")
    with pytest.raises(RuntimeError, match="differs from the build manifest"):
        build.verify_loaded(str(fake))
    other = dict(m, source_digest="0" * 64)
    monkeypatch.setattr(build, "manifest_path", lambda: tmp_path / "m.json")
    (tmp_path / "m.json").write_text(json.dumps(other))
    with pytest.raises(RuntimeError, match="other kernel sources"):
        build.verify_loaded(str(build.so_path()))


def test_digests_do_not_depend_on_where_the_tree_lives(tmp_path, monkeypatch):
    """The GPU box unpacks the tree under another path (and the driver runs smoke() there without
    building): the same sources and flags must give the same object and extension digests, or the
    provenance check would reject a current .so."""
    import shutil

    here = build._plan()
    moved = tmp_path / "elsewhere" / "repo"
    shutil.copytree(build.CSRC, moved / "dstack_amd" / "ops" / "csrc")
    monkeypatch.setattr(build, "ROOT", moved)
    monkeypatch.setattr(build, "HERE", moved / "dstack_amd" / "ops")
    monkeypatch.setattr(build, "CSRC", moved / "dstack_amd" / "ops" / "csrc")
    monkeypatch.setattr(build, "BUILD", moved / "build" / "ops")
    there = build._plan()
    assert str(moved) in " ".join(there[1])  # the commands do name the new location...
    assert [u[2] for u in there[0]] == [u[2] for u in here[0]] and there[2] == here[2]  # ...the digests do not
