#!/bin/bash
# bench A/B only: default + each env variant given as an argument
source "$(dirname "$0")/gpu_tests.sh"
run bench 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile
i=0
for v in "$@"; do
  i=$((i+1))
  run bench_v$i 300 env $v python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile
done
