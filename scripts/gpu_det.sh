#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
run det_fused 300 python tools/determinism.py
run det_fused_single 300 env TAIR_CN_FORK=0 TAIR_ZC_OVERLAP=0 python tools/determinism.py
run det_unfused 300 env TAIR_GN_FUSED=0 python tools/determinism.py
run rocprof_f 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rocprof_f -o f -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-profile
