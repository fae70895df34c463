#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
run rocprof_a 600 env TAIR_CN_FORK=0 TAIR_ZC_OVERLAP=0 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rocprof_a -o a -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile
run rocprof_b 600 env TAIR_GN_FUSED=0 TAIR_CN_FORK=0 TAIR_ZC_OVERLAP=0 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rocprof_b -o b -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile
