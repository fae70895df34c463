#!/bin/bash
# Tile-kernel activation arguments held in registers: GEMM kernel + network tests, then B=1 / B=16 / B=64 lines.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=actargs
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_cldm_gpu.py tests/test_fp8_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_${T}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_${T}_tests.log; [ $rc -eq 0 ] || exit 1
B="--no-cpu-baseline --no-profile --no-stage3-probe"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 $B > gpurun_out/r4_${T}_b1.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --batch 16 --tiles 16 --steps 2 --warmup 1 $B > gpurun_out/r4_${T}_b16.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --batch 64 --tiles 64 --steps 1 --warmup 1 $B > gpurun_out/r4_${T}_b64.log 2>&1 || exit 1
for b in b1 b16 b64; do echo "$b $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r4_${T}_$b.log | head -2 | tr '\n' ' ')"; done
