#!/bin/bash
# kernels, model parity, smoke, bench (no CPU baseline)
source "$(dirname "$0")/gpu_tests.sh"
run kern 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -p no:cacheprovider
run cldm 900 env MIOPEN_FIND_MODE=FAST python -m pytest tests/test_cldm_gpu.py -q -m gpu -x -p no:cacheprovider
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 900 python bench.py --steps 3 --warmup 1 --no-cpu-baseline
