#!/bin/bash
# Per-shape timing of the stride-1 3x3 convs: halo tiles vs the implicit-GEMM tile kernels.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
O=gpurun_out/r4_haloprobe.log
: > $O
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
timeout -k 10 120 python -u tools/conv_probe.py >> $O 2>&1 || exit 1
TAIR_HALO=0 timeout -k 10 120 python -u tools/conv_probe.py >> $O 2>&1 || exit 1
timeout -k 10 120 python -u tools/conv_probe.py --no-epilogue --tag halo_noepi --batch 16 64 >> $O 2>&1 || exit 1
TAIR_HALO=0 timeout -k 10 120 python -u tools/conv_probe.py --no-epilogue --tag tile_noepi --batch 16 64 >> $O 2>&1 || exit 1
for f in 256x64/1/9 256x64/2/9 256x128/1/9 256x128/2/9 256x128/4/9; do
  timeout -k 10 120 python -u tools/conv_probe.py --force $f --tag $f --batch 1 16 >> $O 2>&1 || exit 1
done
