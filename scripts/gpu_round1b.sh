#!/bin/bash
# tests + smoke + bench (with CPU baseline) + rocprof kernel stats
source "$(dirname "$0")/gpu_tests.sh"
TAG=${TAG:-r01}
run kern 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -x -p no:cacheprovider
run cldm 900 python -m pytest tests/test_cldm_gpu.py -q -m gpu -x -p no:cacheprovider
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 900 python bench.py --steps 3 --warmup 1
run rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof -o $TAG -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile
