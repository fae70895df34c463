#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
run b0 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile
run b_devka1 300 env HIP_FORCE_DEV_KERNARG=1 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile
run b_devka0 300 env HIP_FORCE_DEV_KERNARG=0 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile
run b_pc0 300 env DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile
run b_pc1 300 env DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile
run b_s_devka1 300 env TAIR_CN_FORK=0 TAIR_ZC_OVERLAP=0 HIP_FORCE_DEV_KERNARG=1 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile
