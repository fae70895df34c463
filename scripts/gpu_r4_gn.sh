#!/bin/bash
# GroupNorm-on-load (halo plans): kernel tests, network parity, benches for fusion off / conv2 / all.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TAG:-gn2}
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "groupnorm or conv3" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_${T}_kern.log 2>&1; rc=$?; tail -5 gpurun_out/r4_${T}_kern.log; [ $rc -eq 0 ] || exit 1
rm -f gpurun_out/parity.jsonl
TAIR_GN_TRUNK=1 timeout -k 10 400 python -u -m pytest tests/test_cldm_gpu.py -m gpu -q -k "forward_parity_batch2 or restoration_50 or batched_forward" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_${T}_cldm.log 2>&1; echo "cldm rc=$?"; tail -2 gpurun_out/r4_${T}_cldm.log
cp gpurun_out/parity.jsonl gpurun_out/r4_${T}_parity.jsonl
B="--no-cpu-baseline --no-profile --no-stage3-probe"
for v in off conv2 trunk; do
  E="TAIR_GN_FUSE=$([ $v = off ] && echo 0 || echo 1) TAIR_GN_TRUNK=$([ $v = trunk ] && echo 1 || echo 0)"
  env $E timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 $B > gpurun_out/r4_${T}_b1_$v.log 2>&1 || exit 1
  env $E timeout -k 10 300 python -u bench.py --batch 16 --tiles 16 --steps 2 --warmup 1 $B > gpurun_out/r4_${T}_b16_$v.log 2>&1 || exit 1
  env $E timeout -k 10 300 python -u bench.py --batch 64 --tiles 64 --steps 1 --warmup 1 $B > gpurun_out/r4_${T}_b64_$v.log 2>&1 || exit 1
  for b in b1 b16 b64; do echo "$v $b $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r4_${T}_${b}_$v.log | tr '\n' ' ')"; done
done
TAIR_HALO_S2=1 timeout -k 10 120 python -u tools/conv_probe.py --force 256x160/1/9 --tag s2 --batch 16 64 > gpurun_out/r4_${T}_s2_probe.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/conv_probe.py --force 256x160/1/9 --tag s3 --batch 16 64 >> gpurun_out/r4_${T}_s2_probe.log 2>&1 || exit 1
