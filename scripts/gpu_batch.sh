#!/bin/bash
# configs[2]-style batched tiles on one GPU: throughput vs tile batch (MFMA-bound regime)
source "$(dirname "$0")/gpu_tests.sh"
for b in ${BATCHES:-8 32 64}; do
  run bench_b$b 600 python bench.py --steps 1 --warmup 1 --batch $b --no-cpu-baseline
done
