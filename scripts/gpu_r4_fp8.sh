#!/bin/bash
# fp8 layer-set accuracy probe + throughput A/B (bf16 vs fp8) at configs[1] (B=1) and configs[2] (B=64).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step r4_fp8_masks 600 python -u tools/fp8_mask_probe.py 0 16 1 2 4 8 3 31 || exit 1
step r4_bench_b1 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile || exit 1
step r4_bench_b1_fp8 400 python -u bench.py --steps 3 --warmup 1 --fp8 --no-cpu-baseline --no-profile --no-stage3-probe || exit 1
step r4_bench_cfg2 500 python -u bench.py --config 2 --steps 1 --warmup 1 --no-cpu-baseline --no-profile || exit 1
step r4_bench_cfg2_fp8 500 python -u bench.py --config 2 --fp8 --steps 1 --warmup 1 --no-cpu-baseline --no-profile || exit 1
