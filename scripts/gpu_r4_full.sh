#!/bin/bash
# Round-4 checkpoint: smoke(), the whole -m gpu suite, then the bench lines of configs[1] (default), [4], [3] (1 GPU), [2].
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step r4_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
if [ "${SKIP_TESTS-0}" != "1" ]; then
  step r4_pytest_gpu 1100 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider || exit 1
fi
step r4_bench_cfg1 500 python -u bench.py || exit 1
step r4_bench_cfg4 400 python -u bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
step r4_bench_cfg3 900 python -u bench.py --config 3 --steps 1 --warmup 1 --no-cpu-baseline --no-profile || exit 1
step r4_bench_cfg2 600 python -u bench.py --config 2 --steps 1 --warmup 1 --no-cpu-baseline --no-profile || exit 1
