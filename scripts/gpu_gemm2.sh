#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
run kern 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -p no:cacheprovider
run floor 120 python tools/launch_floor.py
run cldm 900 env MIOPEN_FIND_MODE=FAST python -m pytest tests/test_cldm_gpu.py -q -m gpu -x -p no:cacheprovider
run bench 900 python bench.py --steps 3 --warmup 1 --no-cpu-baseline
run gemmsweep 900 python tools/gemm_bench.py gpurun_out/prof_b1.csv --sweep --reps 10 --out gpurun_out/gemm_b1_v4.json
