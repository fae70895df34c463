"""Builds libtair_cldm.so (HIP kernels + C ABI) in-tree for gfx950 with hipcc.

No torch headers are involved: the library exposes only the C ABI of include/tair_cldm.h and
include/tair_kernels.h.  Every translation unit compiles in parallel (the GEMM is split per
activation mode so no unit takes more than ~30 s); objects are rebuilt when their source or any
header under tair_amd/csrc/ or include/ is newer.  `ensure_built()` is what the product calls at
first use: it takes a file lock (several ranks may start at once), rebuilds only when the library
is missing or older than a source, and fails loudly when hipcc is absent.

Usage:  python -m tair_amd.build [--force] [--jobs N]
        python -m tair_amd.build --variant NAME -D MACRO=VALUE ...   (A/B experiments only: builds
        tair_amd/libtair_cldm_NAME.so from the same sources with extra defines; the product never loads
        it -- tools and scripts select it with TAIR_LIB_VARIANT=NAME)
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import fcntl
import glob
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "tair_amd", "csrc")
INCLUDE = os.path.join(ROOT, "include")
BUILD = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(ROOT, "tair_amd", "libtair_cldm.so")
LOCK = os.path.join(ROOT, "tair_amd", ".build.lock")
ARCH = os.environ.get("TAIR_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", CSRC, "-I", INCLUDE,
         "-Wno-unused-result", "-Wno-unused-value", "-munsafe-fp-atomics"]


class BuildError(RuntimeError):
    pass


def sources():
    return sorted(os.path.basename(p) for p in glob.glob(os.path.join(CSRC, "*.hip")) +
                  glob.glob(os.path.join(CSRC, "*.cpp")))


def headers():
    return sorted(glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h")))


def _mtime(p):
    return os.path.getmtime(p)


def _needs(out: str, deps) -> bool:
    if not os.path.exists(out):
        return True
    t = _mtime(out)
    return any(_mtime(d) > t for d in deps)


def is_stale() -> bool:
    """True when the library is missing or older than any source / header."""
    return _needs(LIB, [os.path.join(CSRC, s) for s in sources()] + headers())


def _hipcc():
    if os.path.isfile(HIPCC) and os.access(HIPCC, os.X_OK):
        return HIPCC
    p = shutil.which("hipcc")
    if not p:
        raise BuildError(f"tair_amd: hipcc not found (looked at {HIPCC} and PATH); the HIP library cannot be "
                         "built and there is no CPU fallback")
    return p


def compile_one(src: str, force: bool, hipcc: str, verbose: bool, bdir: str = BUILD, defines=()) -> str:
    path = os.path.join(CSRC, src)
    obj = os.path.join(bdir, src + ".o")
    if force or _needs(obj, [path] + headers()):
        t0 = time.time()
        cmd = [hipcc] + FLAGS + [f"-D{d}" for d in defines] + ["-x", "hip", "-c", path, "-o", obj + ".tmp"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise BuildError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(obj + ".tmp", obj)
        if verbose:
            print(f"[tair_amd.build] {src}: {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    return obj


def source_hash(defines=()) -> str:
    """sha256 (16 hex digits) of every source and header the library is compiled from (paths relative to the
    repo, contents), plus any extra -D defines: the identity of a build, written beside the library
    (`<lib>.srchash`) and into the rocprof / PMC summaries, so a summary can be matched to the code it measured."""
    import hashlib
    h = hashlib.sha256()
    for p in [os.path.join(CSRC, s) for s in sources()] + headers():
        h.update(os.path.relpath(p, ROOT).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    for d in sorted(defines):
        h.update(b"-D" + d.encode() + b"\0")
    return h.hexdigest()[:16]


def library_hash(lib: str = LIB):
    """The source hash recorded when `lib` was built (None if it has no record)."""
    try:
        with open(lib + ".srchash") as f:
            return f.read().strip() or None
    except OSError:
        return None


def variant_lib(name: str) -> str:
    return os.path.join(ROOT, "tair_amd", f"libtair_cldm_{name}.so")


def build(force: bool = False, jobs: int = 0, verbose: bool = True, variant: str = "", defines=()) -> str:
    hipcc = _hipcc()
    bdir = BUILD if not variant else os.path.join(ROOT, "build", f"obj_{variant}")
    lib = LIB if not variant else variant_lib(variant)
    os.makedirs(bdir, exist_ok=True)
    # objects are reused only when built with the same -D set (a variant rebuilt with other defines
    # would otherwise link the previous objects)
    stamp = os.path.join(bdir, "defines.txt")
    want = "\n".join(sorted(defines))
    try:
        with open(stamp) as f:
            force = force or f.read() != want
    except OSError:
        force = force or bool(defines)
    jobs = jobs or min(16, os.cpu_count() or 4)
    t0 = time.time()
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: compile_one(s, force, hipcc, verbose, bdir, defines), srcs))
    with open(stamp, "w") as f:
        f.write(want)
    relinked = force or _needs(lib, objs)
    if relinked:
        tmp = lib + ".tmp"
        cmd = [hipcc, "-shared", f"--offload-arch={ARCH}", "-o", tmp] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise BuildError(f"link failed:\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, lib)
        if verbose:
            print(f"[tair_amd.build] linked {lib} ({len(objs)} objects, {time.time() - t0:.1f}s, "
                  f"{jobs} jobs)", file=sys.stderr, flush=True)
    if relinked or library_hash(lib) is None:
        with open(lib + ".srchash.tmp", "w") as f:
            f.write(source_hash(defines) + "\n")
        os.replace(lib + ".srchash.tmp", lib + ".srchash")
    return lib


def ensure_built(verbose: bool = True) -> str:
    """Build the library if it is missing or stale, under an exclusive file lock."""
    if not is_stale():
        return LIB
    os.makedirs(os.path.dirname(LOCK), exist_ok=True)
    with open(LOCK, "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if is_stale():  # another process may have built it while we waited
                if verbose:
                    print(f"[tair_amd.build] {LIB} missing or stale: building for {ARCH}", file=sys.stderr,
                          flush=True)
                build(verbose=verbose)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=0)
    ap.add_argument("--variant", default="")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    a = ap.parse_args()
    if a.defines and not a.variant:
        ap.error("-D needs --variant (the product library is always built without extra defines)")
    try:
        build(a.force, a.jobs, variant=a.variant, defines=a.defines)
    except BuildError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
