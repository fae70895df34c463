#!/bin/bash
# GroupNorm apply with more rows per block on large grids: kernel + network tests, bandwidth probe, B=64 / B=16 / B=1.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TAG:-gnbw}
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_cldm_gpu.py tests/test_vae_gpu.py -m gpu -x -q -k "not restoration_50" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_${T}_tests.log 2>&1; rc=$?; tail -1 gpurun_out/r4_${T}_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/gn_probe.py --batch 64 > gpurun_out/r4_${T}_probe.log 2>&1 || exit 1
B="--no-cpu-baseline --no-profile --no-stage3-probe"
timeout -k 10 300 python -u bench.py --batch 64 --tiles 64 --steps 1 --warmup 1 $B > gpurun_out/r4_${T}_b64.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --batch 16 --tiles 16 --steps 2 --warmup 1 $B > gpurun_out/r4_${T}_b16.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 $B > gpurun_out/r4_${T}_b1.log 2>&1 || exit 1
for b in b1 b16 b64; do echo "$b $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r4_${T}_$b.log | head -2 | tr '\n' ' ')"; done
