#!/bin/bash
# Round-5: attention variants. Every attention plan at B=64 with the software-pipelined loop (libtair_cldm_pipe1.so; 16 queries
# per wave fits it in 154 VGPRs = 3 waves per SIMD) against the product loop.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-160; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
TAIR_LIB_VARIANT=pipe1 step atests_pipe1 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" || exit 1
step attnb64_main 400 python -u tools/attn_bench.py --batch 64 --reps 5 || exit 1
TAIR_LIB_VARIANT=pipe1 step attnb64_pipe1 400 python -u tools/attn_bench.py --batch 64 --reps 5 || exit 1
# lazy O / l rescale (libtair_cldm_lazy1.so: skipped when no lane's running max moved; bitwise)
TAIR_LIB_VARIANT=lazy1 step atests_lazy1 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or attn" || exit 1
for r in 1 2; do
  step attn_main$r 200 python -u tools/attn_ablate.py --tag main || exit 1
  TAIR_LIB_VARIANT=lazy1 step attn_lazy1_$r 200 python -u tools/attn_ablate.py --tag lazy1 || exit 1
done
