#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
run gemm_b1 600 python tools/gemm_bench.py tools/prof_b1_v0.csv --out gpurun_out/gemm_b1h.json
run bench 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline
run bench8 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch 8
