#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
run b_default 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile
run b_nofork 300 env TAIR_CN_FORK=0 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile
run b_nozc 300 env TAIR_ZC_OVERLAP=0 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile
run b_single 300 env TAIR_CN_FORK=0 TAIR_ZC_OVERLAP=0 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile
run b_single_ik 300 env TAIR_CN_FORK=0 TAIR_ZC_OVERLAP=0 TAIR_SPLITK_INKERNEL=1 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile
run rocprof1 600 env TAIR_CN_FORK=0 TAIR_ZC_OVERLAP=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof_single -o single -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile
