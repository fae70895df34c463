#!/bin/bash
# HIP MSDeformAttn: kernel test + stage-3 tests, then the configs[4] loop bench.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_stage3_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -k "ms_deform or stage3 or testr or graphed or sync" > gpurun_out/r3_msda_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3_msda_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile --config 4 > gpurun_out/r3_msda_cfg4.log 2>&1 || exit $?
python3 -c "import json; r=json.loads(open('gpurun_out/r3_msda_cfg4.log').read().strip().splitlines()[-1]); print('cfg4', r['breakdown_ms']['per_denoise_step_per_micro_batch'], r['value'])"
