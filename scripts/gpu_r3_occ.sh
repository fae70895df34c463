#!/bin/bash
# U = 1 + 4 waves/SIMD on the 2-stage 64x64 tiles: GEMM / model tests, then B=1, B=16, configs[2] bench.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/parity.jsonl
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_cldm_gpu.py tests/test_fp8_gpu.py -x -q -m gpu --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_occ_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r3_occ_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/r3_occ_b1.log 2>&1 || exit $?
python3 -c "import json; r=json.loads(open('gpurun_out/r3_occ_b1.log').read().strip().splitlines()[-1]); print('b1', r['breakdown_ms']['per_denoise_step_per_micro_batch'], r['value'])"
timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --batch 16 --tiles 64 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/r3_occ_b16.log 2>&1 || exit $?
python3 -c "import json; r=json.loads(open('gpurun_out/r3_occ_b16.log').read().strip().splitlines()[-1]); print('b16', r['breakdown_ms']['per_denoise_step_per_micro_batch'], r['value'], r['roofline']['frac'])"
timeout -k 10 600 python -u bench.py --config 2 --steps 1 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/r3_occ_cfg2.log 2>&1 || exit $?
python3 -c "import json; r=json.loads(open('gpurun_out/r3_occ_cfg2.log').read().strip().splitlines()[-1]); print('cfg2', r['breakdown_ms']['per_denoise_step_per_micro_batch'], r['value'], r['roofline']['frac'])"
