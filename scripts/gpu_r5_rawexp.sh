#!/bin/bash
# Round-5: bare v_exp_f32 in the attention softmax vs exp2f (libtair_cldm_oldexp.so): kernel tests, goldens,
# attention timing (interleaved), B=1 and configs[2] step rate.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-160; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step atests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" || exit 1
step golden 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_golden_gpu.py || exit 1
step attn_new 200 python -u tools/attn_ablate.py --tag rawexp || exit 1
TAIR_LIB_VARIANT=oldexp step attn_old 200 python -u tools/attn_ablate.py --tag exp2f || exit 1
step attn_new2 200 python -u tools/attn_ablate.py --tag rawexp || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step b1_new 300 $B || exit 1
TAIR_LIB_VARIANT=oldexp step b1_old 300 $B || exit 1
step b1_new2 300 $B || exit 1
step cfg2_new 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
TAIR_LIB_VARIANT=oldexp step cfg2_old 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
