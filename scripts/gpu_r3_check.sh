#!/bin/bash
# Round-3 re-entry check: fp8 GPU tests, then a B=1 bench.  Stops at the first GPU failure.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_fp8_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_fp8.log 2>&1
rc=$?; echo "fp8 rc=$rc"; tail -15 gpurun_out/r3_fp8.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-stage3-probe > gpurun_out/r3_bench_b1.log 2>&1 || exit $?
tail -1 gpurun_out/r3_bench_b1.log | cut -c1-400
