#!/bin/bash
# In-kernel split-K combine: GEMM kernel tests + forward parity, then B=1 bench A/B over TAIR_INK_SMAX.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/parity.jsonl
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_cldm_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -k "gemm or conv or forward or sampler" > gpurun_out/r3_ink_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3_ink_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for m in ${SMAX:-0 2 3 4}; do
  TAIR_INK_SMAX=$m timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/ink_$m.log 2>&1 || exit $?
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/ink_$m.log').read().strip().splitlines()[-1]); print('ink_smax', $m, r['breakdown_ms']['per_denoise_step_per_micro_batch'], 'ms/step', r['value'])"
done
