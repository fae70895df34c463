#!/bin/bash
# Phase stamps of B=1 GEMM launches (stamps variant library), then the conv_in change's parity + B=1 bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n ${TAILN:-3} "gpurun_out/$name.log" | cut -c1-600; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
TAILN=30 TAIR_LIB_VARIANT=stamps step stamps 300 python -u tools/b1_stamps.py \
  --shapes lin64proj,lin32proj,lin16proj,lin8proj,lin64qkv,lin64ff1,lin16ff2,conv64,conv32,conv16,conv8 \
  --variants plan,e2:plan,halo256x64/s5,halo256x128/s10 || exit 1
step pytest_fwd 600 python -u -m pytest tests/test_cldm_gpu.py -x -q -k "forward_parity or no_control or restoration_50" --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step bench_b1 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
