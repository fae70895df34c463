#!/bin/bash
# Round-5: retuned small-grid plans: graph probe of the changed shapes, B=1 bench x2, kernel + network tests.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step probe_plan 300 python -u tools/b1_probe.py --shapes lin32proj,lin16proj,lin8proj,lin16ff2,lin32ff2,lin16qkv,down32,down16,down8 --variants plan || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step bench_plan1 300 $B || exit 1
step bench_plan2 300 $B || exit 1
step tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_cldm_gpu.py || exit 1
