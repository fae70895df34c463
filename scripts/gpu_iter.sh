#!/bin/bash
# iteration loop: kernel tests, model parity, bench (+ optional A/B env variants given as args)
source "$(dirname "$0")/gpu_tests.sh"
run kern 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -p no:cacheprovider
run cldm 900 python -m pytest tests/test_cldm_gpu.py -q -m "gpu and not slow" -x -p no:cacheprovider
run bench 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile
i=0
for v in "$@"; do
  i=$((i+1))
  run bench_v$i 300 env $v python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile
done
