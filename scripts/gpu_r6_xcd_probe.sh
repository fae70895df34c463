#!/bin/bash
# GEGLU-in 64^2 at B = 64 in isolation under both tile orders (TAIR_XCD=1 m-fastest, 2 n-fastest): time + FETCH_SIZE.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
for x in 1 2; do
  TAIR_XCD=$x timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_xcd$x -o run --output-format csv -- \
    python3 tools/gemm_sweep.py --batch 64 --shapes ${SHAPES:-lin64ff1,lin16ff1} --reps 6 > gpurun_out/pmc_xcd$x.log 2>&1 || exit 1
  echo "TAIR_XCD=$x"; grep shape gpurun_out/pmc_xcd$x.log
  python3 tools/pmc_summary.py /tmp/x$x.json gpurun_out/pmc_xcd$x | grep gemm_tile
done
