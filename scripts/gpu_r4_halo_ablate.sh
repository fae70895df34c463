#!/bin/bash
# Halo conv variants / ablations on one box (timing only, compile-time kernel variants, GemmArgs.probe bits):
# 8 no weight DMA, 16 no MFMA, 32 no loop barrier.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
for rep in 1 2; do
for ab in ${ABL:-0 8 16 24 32 40 56}; do
  for ep in "" "--no-epilogue"; do
    for sh in 64,320,320 32,640,640 16,1280,1280; do
      timeout -k 10 120 python -u tools/conv_probe.py --batch 64 --only $sh --force 256x160/1/9 --ablate $ab --reps 20 \
        --tag "abl$ab$ep" $ep >> gpurun_out/halo_ablate.log 2>&1 || exit 1
    done
  done
done
done
grep '"us"' gpurun_out/halo_ablate.log | cut -c1-130
