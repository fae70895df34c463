#!/bin/bash
# Halo-conv loop change: GEMM kernel tests, conv probe at B=64 (heuristic plans), ablation lines, B=64 / B=16 bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TAG:-halo}
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_${T}_kern.log 2>&1; rc=$?; tail -3 gpurun_out/r4_${T}_kern.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/conv_probe.py --batch 64 --tag $T > gpurun_out/r4_${T}_conv.log 2>&1 || exit 1
tail -1 gpurun_out/r4_${T}_conv.log
for ab in 0 16; do
  for sh in 64,320,320 32,640,640 16,1280,1280; do
    timeout -k 10 120 python -u tools/conv_probe.py --batch 64 --only $sh --force 256x160/1/9 --ablate $ab --reps 10 \
      --tag "${T}_abl${ab}_noepi" --no-epilogue >> gpurun_out/r4_${T}_abl.log 2>&1 || exit 1
  done
done
grep -h '"us"' gpurun_out/r4_${T}_abl.log | cut -c1-120
B="--no-cpu-baseline --no-profile --no-stage3-probe"
timeout -k 10 300 python -u bench.py --batch 64 --tiles 64 --steps 1 --warmup 1 $B > gpurun_out/r4_${T}_b64.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --batch 16 --tiles 16 --steps 2 --warmup 1 $B > gpurun_out/r4_${T}_b16.log 2>&1 || exit 1
for b in b16 b64; do echo "$b $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r4_${T}_$b.log | head -2 | tr '\n' ' ')"; done
