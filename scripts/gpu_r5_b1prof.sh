#!/bin/bash
# tools/b1_probe.py under rocprofv3 --kernel-trace --stats: per-kernel durations (GEMM kernel vs split-K reduce)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
T=${TAG:-b1prof}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$T -o run --output-format csv -- \
  python3 -u tools/b1_probe.py ${SHAPES:+--shapes $SHAPES} ${VARIANTS:+--variants $VARIANTS} --n 20 --reps 2 \
  > gpurun_out/$T.log 2>&1
rc=$?; tail -20 gpurun_out/$T.log; find gpurun_out/$T -name "*kernel_stats.csv" | head -1 | xargs -r cut -c1-160 | head -30; exit $rc
