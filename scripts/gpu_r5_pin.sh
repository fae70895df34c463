#!/bin/bash
# Round-5 paired A/B of the kernel-argument snapshots: product library vs TAIR_PIN=0 ("nopin" variant),
# graph-probe per-launch cost and the B=1 bench step, alternating so box drift hits both sides.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
S=lin64proj,lin32proj,lin16proj,lin16ff2,lin8proj,conv64,conv32,conv16,conv8
step probe_pin 300 python -u tools/b1_probe.py --shapes $S --variants plan || exit 1
TAIR_LIB_VARIANT=nopin step probe_nopin 300 python -u tools/b1_probe.py --shapes $S --variants plan || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step bench_pin1 300 $B || exit 1
TAIR_LIB_VARIANT=nopin step bench_nopin1 300 $B || exit 1
step bench_pin2 300 $B || exit 1
TAIR_LIB_VARIANT=nopin step bench_nopin2 300 $B || exit 1
