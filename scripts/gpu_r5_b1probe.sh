#!/bin/bash
# B=1 per-launch GEMM costs in graph replay (tools/b1_probe.py), variants given in VARIANTS / SHAPES.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
timeout -k 10 900 python -u tools/b1_probe.py ${SHAPES:+--shapes $SHAPES} ${VARIANTS:+--variants $VARIANTS} \
  > gpurun_out/${TAG:-b1probe}.log 2>&1
rc=$?; tail -40 gpurun_out/${TAG:-b1probe}.log; exit $rc
