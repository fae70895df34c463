#!/bin/bash
# fp8 layer sets at B=64 (one 64-tile micro-batch, 50 steps) + the 50-step image gate for a chosen set
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"per_denoise_step_per_micro_batch": [0-9.]*' "gpurun_out/$name.log"; tail -2 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step r4_b64_bf16 300 python -u bench.py --batch 64 --tiles 64 --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-stage3-probe || exit 1
for m in ${MASKS:-16 18 31}; do
  TAIR_FP8_OPS=$m step r4_b64_fp8_$m 300 python -u bench.py --batch 64 --tiles 64 --steps 1 --warmup 1 --fp8 --no-cpu-baseline --no-profile --no-stage3-probe || exit 1
done
TAIR_FP8_OPS=${GATE_MASK:-18} step r4_fp8_gate 600 python -u -m pytest tests/test_fp8_gpu.py -x -q -m gpu --timeout 500 --timeout-method thread -p no:cacheprovider || exit 1
