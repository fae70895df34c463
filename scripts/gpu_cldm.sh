#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
export MIOPEN_FIND_MODE=FAST
run cldm 1100 python -m pytest tests/test_cldm_gpu.py -q -s -m gpu -p no:cacheprovider
cat gpurun_out/parity.jsonl 2>/dev/null
