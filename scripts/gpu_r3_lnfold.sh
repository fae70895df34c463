#!/bin/bash
# LayerNorm folding: GEMM kernel tests + forward/sampler parity + fp8 (unfolded path), then B=1 and
# B=16 bench A/B (TAIR_LN_FOLD=0 vs default).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/parity.jsonl
timeout -k 10 800 python -u -m pytest tests/test_kernels_gpu.py tests/test_cldm_gpu.py tests/test_golden_gpu.py -x -q -m gpu --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_lnf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3_lnf_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for m in 0 1; do
  TAIR_LN_FOLD=$m timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/lnf_$m.log 2>&1 || exit $?
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/lnf_$m.log').read().strip().splitlines()[-1]); print('ln_fold', $m, r['breakdown_ms']['per_denoise_step_per_micro_batch'], 'ms/step', r['value'])"
done
for m in 0 1; do
  TAIR_LN_FOLD=$m timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --batch 16 --tiles 16 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/lnf16_$m.log 2>&1 || exit $?
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/lnf16_$m.log').read().strip().splitlines()[-1]); print('ln_fold b16', $m, r['breakdown_ms']['per_denoise_step_per_micro_batch'], 'ms/step', r['value'])"
done
