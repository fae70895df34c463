#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
TAG=${TAG:-trace}
run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof -o $TAG -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile
