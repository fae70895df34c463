#!/bin/bash
# Round-5: attention at 4 waves per SIMD (launch bounds, 32 VGPRs spilled) vs the product build; timing only
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-160; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step atests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" || exit 1
TAIR_LIB_VARIANT=wpe4 step atests_wpe4 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" || exit 1
for r in 1 2; do
  step attn_main$r 200 python -u tools/attn_ablate.py --tag main || exit 1
  TAIR_LIB_VARIANT=wpe4 step attn_wpe4_$r 200 python -u tools/attn_ablate.py --tag wpe4 || exit 1
done
