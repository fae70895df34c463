#!/bin/bash
# Round-5: attention software pipeline (TAIR_ATTN_PIPE) + scores scaled before the max (TAIR_ATTN_SCALE_FIRST)
# vs libtair_cldm_pipe0.so (scale-first only) and libtair_cldm_r5base.so (neither): kernel tests, goldens,
# attention timing interleaved, B=1 and configs[2].
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-160; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step atests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" || exit 1
step golden 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_golden_gpu.py || exit 1
for r in 1 2; do
  step attn_pipe$r 200 python -u tools/attn_ablate.py --tag pipe || exit 1
  TAIR_LIB_VARIANT=pipe0 step attn_pipe0_$r 200 python -u tools/attn_ablate.py --tag pipe0 || exit 1
  TAIR_LIB_VARIANT=r5base step attn_base$r 200 python -u tools/attn_ablate.py --tag base || exit 1
done
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step b1_pipe 300 $B || exit 1
TAIR_LIB_VARIANT=r5base step b1_base 300 $B || exit 1
step b1_pipe2 300 $B || exit 1
step cfg2_pipe 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
TAIR_LIB_VARIANT=r5base step cfg2_base 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
