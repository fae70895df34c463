#!/bin/bash
# The driver's round-end GPU sequence, from a clean tree (no prebuilt library, no objects):
#   pytest -m gpu, __graft_entry__.smoke(), bench.py --gpus 1 --steps 20 --warmup 5.
# Each step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
rm -rf build tair_amd/libtair_cldm.so
export PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -5 "gpurun_out/$name.log"; return $rc; }
step pytest_gpu 900 python -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider &&
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
step bench 600 python -u bench.py --gpus 1 --steps ${BENCH_STEPS:-20} --warmup ${BENCH_WARMUP:-5}
