#!/bin/bash
# Round-5 A/B: the B=1 tile loop's copy issue interleaved with its fragment reads / MFMAs (product) vs issued
# before them (noilv variant): kernel tests, graph probe of B=1 shapes, B=1 bench x2 each, B=16 bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c90-150; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step ktests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py || exit 1
S=lin64proj,lin32proj,lin16proj,lin8proj,lin16ff2,lin32ff2,conv64,conv32,conv16,conv8
step probe_ilv 300 python -u tools/b1_probe.py --shapes $S --variants plan || exit 1
TAIR_LIB_VARIANT=noilv step probe_noilv 300 python -u tools/b1_probe.py --shapes $S --variants plan || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step b1_ilv 300 $B || exit 1
TAIR_LIB_VARIANT=noilv step b1_noilv 300 $B || exit 1
step b1_ilv2 300 $B || exit 1
TAIR_LIB_VARIANT=noilv step b1_noilv2 300 $B || exit 1
step b16_ilv 300 $B --batch 16 || exit 1
TAIR_LIB_VARIANT=noilv step b16_noilv 300 $B --batch 16 || exit 1
