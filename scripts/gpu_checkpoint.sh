#!/bin/bash
# Round checkpoint: full bench line (with CPU baseline), per-launch profile CSV, rocprofv3 kernel stats.
source "$(dirname "$0")/gpu_tests.sh"
TAG=${TAG:-r01}
run bench 900 python bench.py --steps 3 --warmup 1
TAIR_PROFILE_CSV=gpurun_out/prof_b1.csv run prof1 300 python bench.py --profile-only --batch 1
run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof -o $TAG -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile
