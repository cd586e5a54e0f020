"""Native runtime under sanitizers (host code only): ASan+UBSan and TSan builds of a self-test.

csrc/runtime/tests/selftest.cpp drives the BlockManager (prefix sharing, eviction,
rollback, double free) against a shadow model and the token-FSM compiler against a
naive DFA walk; the TSan build runs the compiler from four threads at once.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(ROOT, "csrc", "runtime")
SRCS = [os.path.join(RT, f) for f in ("block_manager.cpp", "token_fsm.cpp", "tests/selftest.cpp")]


def _build_and_run(tmp_path, flags, mode):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = str(tmp_path / f"selftest_{mode}")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", *flags, *SRCS, "-o", exe, "-pthread"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    proc = subprocess.run([exe, mode], capture_output=True, text=True, timeout=600, env=env)
    assert proc.returncode == 0, proc.stdout + proc.stderr
    assert f"OK {mode}" in proc.stdout


def test_runtime_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"], "asan")


def test_runtime_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], "tsan")
