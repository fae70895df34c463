#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
run kern 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -p no:cacheprovider
run attnbench 300 python tools/attn_bench.py
run cldm 900 env MIOPEN_FIND_MODE=FAST python -m pytest tests/test_cldm_gpu.py -q -m gpu -x -p no:cacheprovider
run bench 900 python bench.py --steps 3 --warmup 1 --no-cpu-baseline
