#!/bin/bash
# Software-pipelined GEMM main loop: kernel tests, conv probe (tile vs halo), B=1 / B=16 / B=64 bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TAG:-pipe}
O=gpurun_out/r4_${T}_probe.log
: > $O
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_${T}_kern.log 2>&1 || { tail -30 gpurun_out/r4_${T}_kern.log; exit 1; }
TAIR_HALO=0 timeout -k 10 120 python -u tools/conv_probe.py --tag tile >> $O 2>&1 || exit 1
for f in 256x128/1/9 256x160/1/9 256x192/1/9 256x160/2/9; do
  timeout -k 10 120 python -u tools/conv_probe.py --force $f --tag $f --batch 16 64 >> $O 2>&1 || exit 1
done
B="--no-cpu-baseline --no-profile --no-stage3-probe"
TAIR_HALO=0 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 $B > gpurun_out/r4_${T}_b1.log 2>&1 || exit 1
TAIR_HALO=0 timeout -k 10 300 python -u bench.py --batch 16 --tiles 16 --steps 2 --warmup 1 $B > gpurun_out/r4_${T}_b16.log 2>&1 || exit 1
TAIR_HALO=0 timeout -k 10 300 python -u bench.py --batch 64 --tiles 64 --steps 1 --warmup 1 $B > gpurun_out/r4_${T}_b64.log 2>&1 || exit 1
