#!/bin/bash
# Round-5: 2-stage 64x64 short-K tiles at 3 waves per SIMD (147 VGPRs, no spills; libtair_cldm_sw3.so) vs the
# 4-wave bound (128 VGPRs, 29 spilled to scratch): kernel tests, short-K probe (interleaved), configs[2], B=16.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-160; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
TAIR_LIB_VARIANT=sw3 step ktests_sw3 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm" || exit 1
for r in 1 2; do
  step sk_w4_$r 300 python -u tools/shortk_probe.py --batch 64 --reps 5 --plans heur || exit 1
  TAIR_LIB_VARIANT=sw3 step sk_w3_$r 300 python -u tools/shortk_probe.py --batch 64 --reps 5 --plans heur || exit 1
done
step cfg2_w4 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
TAIR_LIB_VARIANT=sw3 step cfg2_w3 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
B="python -u bench.py --steps 3 --warmup 1 --batch 16 --no-cpu-baseline --no-stage3-probe --no-profile"
step b16_w4 300 $B || exit 1
TAIR_LIB_VARIANT=sw3 step b16_w3 300 $B || exit 1
