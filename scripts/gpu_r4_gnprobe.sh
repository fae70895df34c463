#!/bin/bash
# Halo conv with / without GroupNorm on load, per shape (B = 16 / 64).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
O=gpurun_out/r4_gnprobe.log
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
TAIR_HALO_S2=1 timeout -k 10 120 python -u tools/conv_probe.py --force 256x160/1/9 --tag plain --batch 16 64 > $O 2>&1 || exit 1
timeout -k 10 120 python -u tools/conv_probe.py --force 256x160/1/9 --tag gn --gn --batch 16 64 >> $O 2>&1 || exit 1
TAIR_HALO_S2=1 timeout -k 10 120 python -u tools/conv_probe.py --force 256x160/1/9 --tag plain_noepi --no-epilogue --batch 64 >> $O 2>&1 || exit 1
timeout -k 10 120 python -u tools/conv_probe.py --force 256x160/1/9 --tag gn_noepi --gn --no-epilogue --batch 64 >> $O 2>&1 || exit 1
rm -f gpurun_out/r4_shortk.log
for b in 16 64; do
  timeout -k 10 200 python -u tools/shortk_probe.py --batch $b >> gpurun_out/r4_shortk.log 2>&1 || exit 1
  timeout -k 10 200 python -u tools/shortk_probe.py --batch $b --no-epilogue >> gpurun_out/r4_shortk.log 2>&1 || exit 1
done
