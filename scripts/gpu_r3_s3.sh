#!/bin/bash
# Stage-3 (TESTR convs as GEMMs): stage-3 GPU tests, the configs[4] loop bench; then the XCD order A/B.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_stage3_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_s3_tests.log 2>&1
rc=$?; echo "stage3 tests rc=$rc"; tail -2 gpurun_out/r3_s3_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile --config 4 > gpurun_out/r3_s3_cfg4.log 2>&1 || exit $?
python3 -c "import json; r=json.loads(open('gpurun_out/r3_s3_cfg4.log').read().strip().splitlines()[-1]); print('cfg4', r['breakdown_ms'], r['value'])"
bash scripts/gpu_r3_xcd.sh
