#!/bin/bash
# The driver's round-end GPU sequence on the prebuilt in-tree library: pytest -m gpu, smoke(), bench.py --gpus 1.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400; return $rc; }
step r6_pytest_gpu 1000 python -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider &&
step r6_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
step r6_bench 600 python -u bench.py --gpus 1 --steps ${BENCH_STEPS:-20} --warmup ${BENCH_WARMUP:-5}
