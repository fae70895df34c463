#!/bin/bash
# Round-5: every tile plan on the batched short-K linears at B=64 (the 64x64 2-stage tiles vs the wider ones).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
timeout -k 10 500 python -u tools/shortk_probe.py --batch 64 --reps 5 > gpurun_out/sk_plans_b64.log 2>&1 || exit 1
