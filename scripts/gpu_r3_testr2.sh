#!/bin/bash
# TESTR launch reductions (shape-constant cache, batch-first MHA, two-stream decoder branches in the
# captured graph): stage-3 GPU tests, then configs[4] bench.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_stage3_gpu.py tests/test_testr_cpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/testr2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/testr2_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/testr2_cfg4.log 2>&1 || exit $?
python3 -c "import json; r=json.loads(open('gpurun_out/testr2_cfg4.log').read().strip().splitlines()[-1]); print('cfg4', r['breakdown_ms'], r['value'])"
