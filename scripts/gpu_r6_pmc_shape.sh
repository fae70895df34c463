#!/bin/bash
# PMC traffic of single GEMM shapes (tools/gemm_sweep.py, planner's plan only): FETCH_SIZE and WRITE_SIZE passes.
# SHAPES="lin64ff1,conv8" BATCH=64 TAG=name; output gpurun_out/pmc_${TAG}_{fetch,write}/ + the sweep log.
set -o pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
CMD="python3 tools/gemm_sweep.py --batch ${BATCH:-64} --shapes ${SHAPES} --reps 6"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${TAG}_fetch -o run --output-format csv -- $CMD > gpurun_out/pmc_${TAG}_fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${TAG}_write -o run --output-format csv -- $CMD > gpurun_out/pmc_${TAG}_write.log 2>&1 || exit 1
grep shape gpurun_out/pmc_${TAG}_fetch.log
