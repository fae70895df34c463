#!/bin/bash
# Round-5: the B=64 sampler parity test on the product library (wide short-K plans off).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cldm_gpu.py -k "batch64" > gpurun_out/p64_main.log 2>&1; echo "main rc=$?"
