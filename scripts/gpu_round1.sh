#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
rocm-smi --showproductname > gpurun_out/smi.log 2>&1 || true
run kernels 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -p no:cacheprovider
run cldm 900 python -m pytest tests/test_cldm_gpu.py -q -m "gpu and not slow" -x -p no:cacheprovider
