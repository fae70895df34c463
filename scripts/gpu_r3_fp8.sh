#!/bin/bash
# fp8 (configs[4]) on the GPU: kernel + model tests, then B=1 bench lines with and without fp8 and a
# short configs[4] prompt-loop run.  Stops at the first GPU failure.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/parity.jsonl
timeout -k 10 700 python -u -m pytest tests/test_fp8_gpu.py -x -v -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_fp8.log 2>&1
rc=$?; echo "fp8 rc=$rc"; tail -5 gpurun_out/r3_fp8.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-stage3-probe --fp8 > gpurun_out/r3_bench_b1_fp8.log 2>&1 || exit $?
tail -1 gpurun_out/r3_bench_b1_fp8.log | cut -c1-300
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile --config 4 > gpurun_out/r3_bench_cfg4.log 2>&1 || exit $?
tail -1 gpurun_out/r3_bench_cfg4.log | cut -c1-300
