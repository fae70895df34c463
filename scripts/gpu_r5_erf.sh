#!/bin/bash
# Round-5 A/B: GEGLU epilogue erf (A&S 7.1.26 with hardware rcp / exp, product) vs the library erff (ocmlerf
# variant): short-K probe of the B=64 GEGLU-in shapes, configs[2], the GEGLU / cooperative-split kernel tests.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c90-150; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step ktests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "geglu or cooperative or dense" || exit 1
step sk_fast 300 python -u tools/shortk_probe.py --batch 64 --plans heur || exit 1
TAIR_LIB_VARIANT=ocmlerf step sk_ocml 300 python -u tools/shortk_probe.py --batch 64 --plans heur || exit 1
step cfg2_fast 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
TAIR_LIB_VARIANT=ocmlerf step cfg2_ocml 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
