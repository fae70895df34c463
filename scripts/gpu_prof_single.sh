#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
TAIR_CN_FORK=0 TAIR_ZC_OVERLAP=0 TAIR_PROFILE_CSV=gpurun_out/prof_single.csv run prof1 300 python bench.py --profile-only --batch 1
