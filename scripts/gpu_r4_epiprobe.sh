#!/bin/bash
# Where the short-K epilogue time goes: full / values formed but not stored / no epilogue (B = 64).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
O=gpurun_out/r4_epiprobe.log
: > $O
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
for pr in 0 1 2; do
  timeout -k 10 200 python -u tools/shortk_probe.py --batch 64 --probe $pr --plans heur,64x64/1/2,256x128/1/3 >> $O 2>&1 || exit 1
done
