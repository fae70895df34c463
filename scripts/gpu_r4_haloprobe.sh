#!/bin/bash
# Halo conv tiles: kernel tests, then per-shape timing vs the implicit-GEMM tile kernels, then a B=1
# per-launch table.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
O=gpurun_out/r4_haloprobe.log
: > $O
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "conv3" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_halo_kern2.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/conv_probe.py >> $O 2>&1 || exit 1
TAIR_HALO=0 timeout -k 10 120 python -u tools/conv_probe.py >> $O 2>&1 || exit 1
timeout -k 10 120 python -u tools/conv_probe.py --no-epilogue --tag halo_noepi --batch 16 64 >> $O 2>&1 || exit 1
TAIR_HALO=0 timeout -k 10 120 python -u tools/conv_probe.py --no-epilogue --tag tile_noepi --batch 16 64 >> $O 2>&1 || exit 1
for f in 256x128/1/9 256x160/1/9 256x192/1/9 256x64/2/9 256x128/2/9 256x160/2/9 256x160/4/9; do
  timeout -k 10 120 python -u tools/conv_probe.py --force $f --tag $f --batch 1 16 64 >> $O 2>&1 || exit 1
done
TAIR_PROFILE_CSV=gpurun_out/r4_b1_launches.csv timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-stage3-probe > gpurun_out/r4_b1_launches.log 2>&1 || exit 1
