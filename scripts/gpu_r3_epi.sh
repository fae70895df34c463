#!/bin/bash
# Epilogue operand prefetch: GEMM kernel tests, short-K probe at B=16, B=1 / B=16 bench.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -k "not restoration" > gpurun_out/r3_epi_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r3_epi_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python3 tools/gemm_probe.py --batch 16 --reps 10 --tiles "0x0,e1:0x0,e2:0x0" > gpurun_out/r3_epi_probe_b16.log 2>&1 || exit $?
cat gpurun_out/r3_epi_probe_b16.log
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/r3_epi_b1.log 2>&1 || exit $?
python3 -c "import json; r=json.loads(open('gpurun_out/r3_epi_b1.log').read().strip().splitlines()[-1]); print('b1', r['breakdown_ms']['per_denoise_step_per_micro_batch'], r['value'])"
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --batch 16 --tiles 64 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/r3_epi_b16.log 2>&1 || exit $?
python3 -c "import json; r=json.loads(open('gpurun_out/r3_epi_b16.log').read().strip().splitlines()[-1]); print('b16', r['breakdown_ms']['per_denoise_step_per_micro_batch'], r['value'])"
