#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
run kernels 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -p no:cacheprovider
run gemm_b1 900 python tools/gemm_bench.py tools/prof_b1_v0.csv --sweep --reps 9 --out gpurun_out/gemm_b1_v3.json
