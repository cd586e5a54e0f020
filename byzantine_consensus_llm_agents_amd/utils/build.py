"""In-tree native builds (no pip install, no JIT cache outside the repo).

* ``build_runtime``: C++17 host runtime (``csrc/runtime/*.cpp``) -> pybind11
  module ``runtime/_bcg_runtime*.so`` (g++).
* ``build_kernels``: HIP/CDNA4 kernels (``csrc/kernels/*.hip``) ->
  ``ops/libbcg_kernels.so`` with ``hipcc --offload-arch=gfx950``; a plain C ABI
  loaded through ctypes, so the kernels need no PyTorch headers and build in
  seconds.  Both outputs sit inside the package so they travel to the GPU box
  with the repo snapshot.

Builds are skipped when the output is newer than every source and was built
with the same flags (a ``.flags`` sidecar beside it); concurrent builders (DP
ranks) write to a temp file and ``os.replace`` it into place.

``BCG_EXTRA_HIPFLAGS`` (variant builds for A/B tools, e.g. ``-DPREFILL_LDS_BUILD=1``)
never touches the production library: the variant goes to
``build/libbcg_<hash of the flags>.so`` and is selected with ``BCG_KERNELS_LIB``.
"""

import glob
import hashlib
import os
import subprocess
import sys
import sysconfig
import tempfile

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(REPO, "csrc")
ARCH = os.environ.get("BCG_OFFLOAD_ARCH", "gfx950")


def runtime_target() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "runtime", "_bcg_runtime" + suffix)


def kernels_target() -> str:
    return os.path.join(PKG, "ops", "libbcg_kernels.so")


def variant_target(flags: str) -> str:
    """Where a build with extra hipcc flags goes (never the production library)."""
    tag = hashlib.sha1(" ".join(flags.split()).encode()).hexdigest()[:12]
    return os.path.join(REPO, "build", f"libbcg_{tag}.so")


def _stale(target: str, sources, flags: str = "") -> bool:
    if not os.path.exists(target):
        return True
    stamp = target + ".flags"
    recorded = open(stamp).read() if os.path.exists(stamp) else ""
    if recorded != flags:  # built with other flags: rebuild
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _write_stamp(target: str, flags: str):
    if flags or os.path.exists(target + ".flags"):
        with open(target + ".flags", "w") as fh:
            fh.write(flags)


def _run(cmd):
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"build failed ({proc.returncode}): {' '.join(cmd)}\n{proc.stdout}")
    return proc.stdout


def build_runtime(force: bool = False, verbose: bool = False) -> str:
    import pybind11
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.h")))
    target = runtime_target()
    if not force and not _stale(target, srcs + hdrs):
        return target
    fd, tmp = tempfile.mkstemp(suffix=".so", dir=os.path.dirname(target))
    os.close(fd)
    cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden",
           f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
           f"-I{os.path.join(CSRC, 'runtime')}", *srcs, "-o", tmp]
    out = _run(cmd)
    if verbose and out:
        print(out)
    os.chmod(tmp, 0o755)
    os.replace(tmp, target)
    return target


def build_kernels(force: bool = False, verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")))
    extra = " ".join(os.environ.get("BCG_EXTRA_HIPFLAGS", "").split())
    target = variant_target(extra) if extra else kernels_target()
    os.makedirs(os.path.dirname(target), exist_ok=True)
    if not srcs:
        raise RuntimeError("no HIP kernel sources found")
    if not force and not _stale(target, srcs + hdrs, extra):
        return target
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    fd, tmp = tempfile.mkstemp(suffix=".so", dir=os.path.dirname(target))
    os.close(fd)
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
           "-fgpu-flush-denormals-to-zero", "-munsafe-fp-atomics",
           f"-I{os.path.join(CSRC, 'kernels')}", *srcs, "-o", tmp]
    if os.environ.get("BCG_RESOURCE_USAGE"):
        cmd.insert(1, "-Rpass-analysis=kernel-resource-usage")
    if extra:  # variant builds (tools), e.g. -DPREFILL_LDS_BUILD=1: a separate target
        cmd[1:1] = extra.split()
    out = _run(cmd)
    if verbose and out:
        print(out)
    os.chmod(tmp, 0o755)
    os.replace(tmp, target)
    _write_stamp(target, extra)
    return target


def build_all(force: bool = False, verbose: bool = False):
    return build_runtime(force, verbose), build_kernels(force, verbose)


if __name__ == "__main__":
    for path in build_all(force="--force" in sys.argv, verbose=True):
        print("built", path)
