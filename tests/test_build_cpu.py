"""Native build bookkeeping (utils/build.py): variant flags never reach the production library,
staleness is decided by a hash of the sources (not mtimes), a failed build leaves no temp files,
and a library whose embedded source stamp differs from the tree is refused."""
import ctypes
import glob
import os
import shutil
import subprocess

import pytest

from byzantine_consensus_llm_agents_amd.utils import build


def test_variant_target_is_separate():
    prod = build.kernels_target()
    a = build.variant_target("-DPREFILL_LDS_BUILD=1")
    b = build.variant_target("-DPREFILL_LDS_BUILD=1  ")  # whitespace-normalised: same target
    c = build.variant_target("-DW4_DBS=2")
    assert a != prod and c != prod and a == b and a != c
    assert os.path.basename(a).startswith("libbcg_") and a.endswith(".so")


def test_source_hash_tracks_content(tmp_path):
    a, b = tmp_path / "a.hip", tmp_path / "b.h"
    a.write_text("x")
    b.write_text("y")
    h0 = build.source_hash([str(a), str(b)])
    assert h0 == build.source_hash([str(b), str(a)])          # order-independent
    os.utime(a, None)
    assert build.source_hash([str(a), str(b)]) == h0           # mtime alone: same
    a.write_text("x2")
    assert build.source_hash([str(a), str(b)]) != h0


def test_stale_tracks_hash_and_flags(tmp_path):
    tgt = tmp_path / "lib.so"
    assert build._stale(str(tgt), "h1", "")                     # missing
    tgt.write_text("x")
    assert build._stale(str(tgt), "h1", "")                     # no stamp
    build._write_stamp(str(tgt), "h1", "-DX=1")
    assert build._stale(str(tgt), "h1", "")                     # built with flags, asked without
    assert not build._stale(str(tgt), "h1", "-DX=1")
    assert build._stale(str(tgt), "h2", "-DX=1")                # other sources
    build._write_stamp(str(tgt), "h1", "")
    assert not build._stale(str(tgt), "h1", "")


def test_failed_kernel_build_leaves_no_temp(tmp_path, monkeypatch):
    """A compile error removes the mkstemp target and the object dir (ops/tmp*.so leak)."""
    fake = tmp_path / "hipcc"
    fake.write_text("#!/bin/sh\necho broken source >&2\nexit 1\n")
    fake.chmod(0o755)
    monkeypatch.setenv("HIPCC", str(fake))
    monkeypatch.setenv("BCG_EXTRA_HIPFLAGS", "-DBCG_TEST_FAILED_BUILD=1")
    target = build.variant_target("-DBCG_TEST_FAILED_BUILD=1")
    before = set(os.listdir(os.path.dirname(target))) if os.path.isdir(os.path.dirname(target)) else set()
    with pytest.raises(RuntimeError, match="build failed"):
        build.build_kernels(force=True)
    after = set(os.listdir(os.path.dirname(target)))
    assert after - before == set()


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_mismatched_library_is_refused(tmp_path):
    """ops/hip.py refuses a library whose bcg_source_hash() is not the tree's hash, and one without a stamp."""
    from byzantine_consensus_llm_agents_amd.ops import hip
    good, bad, none = (tmp_path / n for n in ("good.so", "bad.so", "none.so"))
    want = build.kernels_source_hash()
    for path, body in ((good, f'const char* bcg_source_hash(void) {{ return "{want}"; }}'),
                       (bad, 'const char* bcg_source_hash(void) { return "0123456789abcdef"; }'),
                       (none, 'int bcg_other(void) { return 0; }')):
        src = tmp_path / (path.stem + ".c")
        src.write_text(body + "\n")
        subprocess.run(["gcc", "-shared", "-fPIC", str(src), "-o", str(path)], check=True)
    hip.check_source_stamp(ctypes.CDLL(str(good)), str(good))
    with pytest.raises(hip.StaleLibraryError, match="0123456789abcdef"):
        hip.check_source_stamp(ctypes.CDLL(str(bad)), str(bad))
    with pytest.raises(hip.StaleLibraryError, match="None"):
        hip.check_source_stamp(ctypes.CDLL(str(none)), str(none))


def test_built_library_carries_tree_stamp():
    """The in-tree library (when built) is stamped with the current sources."""
    from byzantine_consensus_llm_agents_amd.ops import hip
    path = build.kernels_target()
    if not os.path.exists(path):
        pytest.skip("library not built")
    stamp = hip.library_stamp(ctypes.CDLL(path))
    assert stamp == open(path + ".srchash").read()  # the build's own record of what it compiled
    if stamp != build.kernels_source_hash():  # sources edited since: load_library refuses it
        with pytest.raises(hip.StaleLibraryError):
            hip.check_source_stamp(ctypes.CDLL(path), path)


def test_runtime_module_stamp():
    from byzantine_consensus_llm_agents_amd import runtime
    assert runtime._native.source_hash == build.runtime_source_hash()
