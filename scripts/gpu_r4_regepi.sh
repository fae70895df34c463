#!/bin/bash
# Register-direct epilogue: kernel + network tests, short-K probe (registers vs LDS-staged, probe bit 3),
# B=1 / B=16 / B=64 lines.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TAG:-regepi}
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_cldm_gpu.py tests/test_vae_gpu.py tests/test_fp8_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_${T}_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r4_${T}_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4_${T}_tests.log | head -20; exit 1; }
O=gpurun_out/r4_${T}_probe.log
: > $O
for pr in 0 8; do
  timeout -k 10 200 python -u tools/shortk_probe.py --batch 64 --probe $pr --plans heur,64x64/1/2,256x128/1/3,128x320/1/2 >> $O 2>&1 || exit 1
done
B="--no-cpu-baseline --no-profile --no-stage3-probe"
timeout -k 10 300 python -u bench.py --batch 64 --tiles 64 --steps 1 --warmup 1 $B > gpurun_out/r4_${T}_b64.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --batch 16 --tiles 16 --steps 2 --warmup 1 $B > gpurun_out/r4_${T}_b16.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 $B > gpurun_out/r4_${T}_b1.log 2>&1 || exit 1
for b in b1 b16 b64; do echo "$b $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r4_${T}_$b.log | head -2 | tr '\n' ' ')"; done
