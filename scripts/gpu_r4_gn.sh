#!/bin/bash
# GroupNorm-on-load: kernel tests, network parity (conv2 fused; + residual-stream inputs fused, hi plane),
# then B=1 / B=16 benches for GN fusion off / conv2 / all.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "groupnorm_on_load or conv3" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_gn_kern.log 2>&1; rc=$?; tail -25 gpurun_out/r4_gn_kern.log; [ $rc -eq 0 ] || exit 1
K="forward_parity_batch2 or restoration_50 or sampler_graph or batched_forward"
for v in conv2 trunk; do
  rm -f gpurun_out/parity.jsonl
  TAIR_GN_TRUNK=$([ $v = trunk ] && echo 1 || echo 0) timeout -k 10 400 python -u -m pytest tests/test_cldm_gpu.py -m gpu -q -k "$K" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_gn_cldm_$v.log 2>&1; echo "cldm $v rc=$?"; tail -2 gpurun_out/r4_gn_cldm_$v.log
  cp gpurun_out/parity.jsonl gpurun_out/r4_gn_parity_$v.jsonl
done
B="--no-cpu-baseline --no-profile --no-stage3-probe"
for v in off conv2 trunk; do
  E="TAIR_GN_FUSE=$([ $v = off ] && echo 0 || echo 1) TAIR_GN_TRUNK=$([ $v = trunk ] && echo 1 || echo 0)"
  env $E timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 $B > gpurun_out/r4_gn_b1_$v.log 2>&1 || exit 1
  env $E timeout -k 10 300 python -u bench.py --batch 16 --tiles 16 --steps 2 --warmup 1 $B > gpurun_out/r4_gn_b16_$v.log 2>&1 || exit 1
  for b in b1 b16; do echo "$v $b $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r4_gn_${b}_$v.log | tr '\n' ' ')"; done
done
