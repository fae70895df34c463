#!/bin/bash
# Round-5 A/B: compact epilogue items loop (efast variant, TAIR_EPI_FAST=1) vs product, graph probe + B=1 bench,
# and the kernel tests on the variant.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
S=lin64proj,lin32proj,lin16proj,lin8proj,lin16ff2,conv64,conv16
step probe_base 300 python -u tools/b1_probe.py --shapes $S --variants plan,e1:plan,e2:plan || exit 1
TAIR_LIB_VARIANT=efast step probe_efast 300 python -u tools/b1_probe.py --shapes $S --variants plan || exit 1
TAIR_LIB_VARIANT=efast step tests_efast 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step bench_base 300 $B || exit 1
TAIR_LIB_VARIANT=efast step bench_efast 300 $B || exit 1
