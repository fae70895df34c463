#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
TAG=${TAG:-t}
run rocprof_s 600 env TAIR_CN_FORK=0 TAIR_ZC_OVERLAP=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof_s -o s -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile
run rocprof_f 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof_f -o f -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile
