#!/bin/bash
# Parity tests (fp32 oracle on MIOpen: FAST find mode keeps its first-call tuning short), smoke, bench.
# The bench runs WITHOUT MIOPEN_FIND_MODE=FAST: that mode picks heuristic kernels for the bf16 VAE.
source "$(dirname "$0")/gpu_tests.sh"
run cldm 900 env MIOPEN_FIND_MODE=FAST python -m pytest tests/test_cldm_gpu.py -q -m gpu -x -p no:cacheprovider
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline
