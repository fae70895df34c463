#!/bin/bash
# Round-5: weight-stationary persistent short-K kernel (product) vs the 2-stage 64x64 tiles (TAIR_WRES=0):
# kernel tests, short-K probe at B=64, B=16 and configs[2] A/B, network tests.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c90-150; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step ktests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "weight_stationary or dense or geglu" || exit 1
step sk_wres 300 python -u tools/shortk_probe.py --batch 64 --plans heur || exit 1
TAIR_WRES=0 step sk_nowres 300 python -u tools/shortk_probe.py --batch 64 --plans heur || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step b16_wres 300 $B --batch 16 || exit 1
TAIR_WRES=0 step b16_nowres 300 $B --batch 16 || exit 1
step cfg2_wres 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
TAIR_WRES=0 step cfg2_nowres 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
step ctests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_cldm_gpu.py || exit 1
