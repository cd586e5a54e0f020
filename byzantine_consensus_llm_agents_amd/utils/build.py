"""In-tree native builds (no pip install, no JIT cache outside the repo).

* ``build_runtime``: C++17 host runtime (``csrc/runtime/*.cpp``) -> pybind11
  module ``runtime/_bcg_runtime*.so`` (g++).
* ``build_kernels``: HIP/CDNA4 kernels (``csrc/kernels/*.hip``) ->
  ``ops/libbcg_kernels.so`` with ``hipcc --offload-arch=gfx950``; a plain C ABI
  loaded through ctypes, so the kernels need no PyTorch headers and build in
  seconds.  Both outputs sit inside the package so they travel to the GPU box
  with the repo snapshot.

Both libraries carry a hash of their sources (``source_hash``): the kernels
library exports ``bcg_source_hash()`` and the runtime module a ``source_hash``
attribute.  ``ops/hip.py`` and ``runtime/__init__.py`` compare it with the tree
they are loaded from and refuse a mismatch, so a stale binary shipped next to
newer sources never runs.  Builds are skipped when the recorded hash and flags
(``.srchash`` / ``.flags`` sidecars) match; concurrent builders (DP ranks) write
to a temp file and ``os.replace`` it into place, and a failed build removes its
temp files.  HIP sources compile one process per file, then link.

``BCG_EXTRA_HIPFLAGS`` (variant builds for A/B tools, e.g. ``-DPREFILL_LDS_BUILD=1``)
never touches the production library: the variant goes to
``build/libbcg_<hash of the flags>.so`` and is selected with ``BCG_KERNELS_LIB``.
"""

import glob
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
import tempfile
from concurrent.futures import ThreadPoolExecutor

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


def kernel_sources():
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")))
    return srcs, hdrs


def runtime_sources():
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.h")))
    return srcs, hdrs


def source_hash(paths) -> str:
    """16-hex sha256 over (basename, bytes) of every source, in sorted order."""
    h = hashlib.sha256()
    for p in sorted(paths, key=os.path.basename):
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def kernels_source_hash() -> str:
    srcs, hdrs = kernel_sources()
    return source_hash(srcs + hdrs)


def runtime_source_hash() -> str:
    srcs, hdrs = runtime_sources()
    return source_hash(srcs + hdrs)


def _read(path: str) -> str:
    return open(path).read() if os.path.exists(path) else ""


def _stale(target: str, digest: str, flags: str = "") -> bool:
    """A build is current iff the target exists and was built from sources with
    this hash and with these flags (sidecars written by the build)."""
    if not os.path.exists(target):
        return True
    return _read(target + ".srchash") != digest or _read(target + ".flags") != flags


def _write_stamp(target: str, digest: str, flags: str):
    with open(target + ".srchash", "w") as fh:
        fh.write(digest)
    with open(target + ".flags", "w") as fh:
        fh.write(flags)


def _run(cmd):
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if proc.returncode != 0:
        raise RuntimeError(f"build failed ({proc.returncode}): {' '.join(cmd)}\n{proc.stdout}")
    return proc.stdout


def _cleanup(*paths):
    for p in paths:
        if os.path.isdir(p):
            shutil.rmtree(p, ignore_errors=True)
        elif os.path.exists(p):
            os.remove(p)


def build_runtime(force: bool = False, verbose: bool = False) -> str:
    import pybind11
    srcs, hdrs = runtime_sources()
    digest = source_hash(srcs + hdrs)
    target = runtime_target()
    if not force and not _stale(target, digest):
        return target
    fd, tmp = tempfile.mkstemp(suffix=".so", dir=os.path.dirname(target))
    os.close(fd)
    cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden",
           f'-DBCG_SOURCE_HASH="{digest}"',
           f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
           f"-I{os.path.join(CSRC, 'runtime')}", *srcs, "-o", tmp]
    try:
        out = _run(cmd)
        if verbose and out:
            print(out)
        os.chmod(tmp, 0o755)
        os.replace(tmp, target)
    finally:
        _cleanup(tmp)
    _write_stamp(target, digest, "")
    return target


def build_kernels(force: bool = False, verbose: bool = False) -> str:
    srcs, hdrs = kernel_sources()
    digest = source_hash(srcs + hdrs)
    extra = " ".join(os.environ.get("BCG_EXTRA_HIPFLAGS", "").split())
    target = variant_target(extra) if extra else kernels_target()
    os.makedirs(os.path.dirname(target), exist_ok=True)
    if not srcs:
        raise RuntimeError("no HIP kernel sources found")
    if not force and not _stale(target, digest, extra):
        return target
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    fd, tmp = tempfile.mkstemp(suffix=".so", dir=os.path.dirname(target))
    os.close(fd)
    objdir = tempfile.mkdtemp(prefix="bcg_obj_", dir=os.path.dirname(target))
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
             "-fgpu-flush-denormals-to-zero", "-munsafe-fp-atomics",
             f'-DBCG_SOURCE_HASH="{digest}"', f"-I{os.path.join(CSRC, 'kernels')}"]
    if os.environ.get("BCG_RESOURCE_USAGE"):
        flags.insert(0, "-Rpass-analysis=kernel-resource-usage")
    if extra:  # variant builds (tools), e.g. -DPREFILL_LDS_BUILD=1: a separate target
        flags[0:0] = extra.split()
    objs = [os.path.join(objdir, os.path.basename(s) + ".o") for s in srcs]
    jobs = max(1, min(len(srcs), int(os.environ.get("MAX_JOBS", "0") or 0) or (os.cpu_count() or 1), 16))
    try:
        with ThreadPoolExecutor(jobs) as pool:  # one hipcc per file: gemm_w4 dominates
            outs = list(pool.map(lambda so: _run([hipcc, *flags, "-c", so[0], "-o", so[1]]), zip(srcs, objs)))
        outs.append(_run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp]))
        if verbose:
            print("".join(o for o in outs if o))
        os.chmod(tmp, 0o755)
        os.replace(tmp, target)
    finally:
        _cleanup(tmp, objdir)
    _write_stamp(target, digest, extra)
    return target


def build_all(force: bool = False, verbose: bool = False):
    return build_runtime(force, verbose), build_kernels(force, verbose)


if __name__ == "__main__":
    for path in build_all(force="--force" in sys.argv, verbose=True):
        print("built", path)
