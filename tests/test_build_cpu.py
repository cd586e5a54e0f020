"""Native build bookkeeping (utils/build.py): variant flags never reach the production library,
and a library built with other flags counts as stale (build.py item)."""
import os
import time

from byzantine_consensus_llm_agents_amd.utils import build


def test_variant_target_is_separate():
    prod = build.kernels_target()
    a = build.variant_target("-DPREFILL_LDS_BUILD=1")
    b = build.variant_target("-DPREFILL_LDS_BUILD=1  ")  # whitespace-normalised: same target
    c = build.variant_target("-DW4_DBS=2")
    assert a != prod and c != prod and a == b and a != c
    assert os.path.basename(a).startswith("libbcg_") and a.endswith(".so")


def test_stale_tracks_flags(tmp_path):
    src = tmp_path / "k.hip"
    src.write_text("//")
    old = time.time() - 100
    os.utime(src, (old, old))
    tgt = tmp_path / "lib.so"
    tgt.write_text("x")
    assert not build._stale(str(tgt), [str(src)], "")          # no stamp, no flags: fresh
    build._write_stamp(str(tgt), "-DX=1")
    assert build._stale(str(tgt), [str(src)], "")              # built with flags, asked without
    assert not build._stale(str(tgt), [str(src)], "-DX=1")
    build._write_stamp(str(tgt), "")                           # rebuilt plain: stamp cleared
    assert not build._stale(str(tgt), [str(src)], "")
    os.utime(src, None)                                        # a newer source: stale
    assert build._stale(str(tgt), [str(src)], "")
