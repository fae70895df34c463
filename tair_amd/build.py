"""Builds libtair_cldm.so (HIP kernels + C ABI) in-tree for gfx950 with hipcc.

No torch headers are involved: the library exposes only the C ABI of include/tair_cldm.h.
Usage:  python -m tair_amd.build [--force] [--jobs N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "tair_amd", "csrc")
INCLUDE = os.path.join(ROOT, "include")
BUILD = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(ROOT, "tair_amd", "libtair_cldm.so")
SOURCES = ["gemm.hip", "norm.hip", "attention.hip", "misc.hip", "cldm.cpp", "kapi.cpp"]
ARCH = os.environ.get("TAIR_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", CSRC, "-I", INCLUDE,
         "-Wno-unused-result", "-munsafe-fp-atomics"]


def _needs(obj: str, deps) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs.append(os.path.join(INCLUDE, "tair_cldm.h"))
    return hs


def compile_one(src: str, force: bool) -> str:
    path = os.path.join(CSRC, src)
    obj = os.path.join(BUILD, src + ".o")
    if force or _needs(obj, [path] + _headers()):
        lang = ["-x", "hip"]
        cmd = [HIPCC] + FLAGS + lang + ["-c", path, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int = 4, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: compile_one(s, force), SOURCES))
    if force or _needs(LIB, objs):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[tair_amd.build] {LIB}")
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    a = ap.parse_args()
    try:
        build(a.force, a.jobs)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
