#!/bin/bash
# Round-5: cooperative split-K combine. Kernel tests first (bounded), then the graph probe with/without
# (TAIR_COOP=0), B=1 bench A/B, the network tests.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step ktests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py || exit 1
S=lin32proj,lin16proj,lin8proj,lin16ff2,lin32ff2,conv64,conv32,conv16,conv8,down8,up16,conv16in
step probe_coop 300 python -u tools/b1_probe.py --shapes $S --variants plan || exit 1
TAIR_COOP=0 step probe_nocoop 300 python -u tools/b1_probe.py --shapes $S --variants plan || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step bench_coop1 300 $B || exit 1
TAIR_COOP=0 step bench_nocoop1 300 $B || exit 1
step bench_coop2 300 $B || exit 1
TAIR_COOP=0 step bench_nocoop2 300 $B || exit 1
step ctests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cldm_gpu.py || exit 1
