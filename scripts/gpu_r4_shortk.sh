#!/bin/bash
# Batched short-K linears: heuristic plan vs forced tiles, with and without the epilogue (B = 16 / 64).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
O=gpurun_out/r4_shortk.log
: > $O
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
for b in 16 64; do
  timeout -k 10 200 python -u tools/shortk_probe.py --batch $b >> $O 2>&1 || exit 1
  timeout -k 10 200 python -u tools/shortk_probe.py --batch $b --no-epilogue >> $O 2>&1 || exit 1
done
