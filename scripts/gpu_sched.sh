#!/bin/bash
# schedules of the step graph: grouped vs forked ControlNet, zero convs overlapped or not
source "$(dirname "$0")/gpu_tests.sh"
run cldm 900 env MIOPEN_FIND_MODE=FAST python -m pytest tests/test_cldm_gpu.py -q -m gpu -x -p no:cacheprovider
run b_grp_zc 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile
TAIR_ZC_OVERLAP=0 run b_grp 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile
TAIR_CN_FORK=1 run b_fork_zc 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile
TAIR_CN_FORK=0 run cldm_grp 900 env MIOPEN_FIND_MODE=FAST python -m pytest tests/test_cldm_gpu.py -q -m gpu -x -p no:cacheprovider -k "not 50"
