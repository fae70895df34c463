#!/bin/bash
# Round-5: where the attention kernel's time goes (ablation builds, timing only).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
timeout -k 10 200 python -u tools/attn_ablate.py --tag product > gpurun_out/attn_abl.log 2>&1 || exit 1
for v in 1 4 10 14; do
  TAIR_LIB_VARIANT=abl$v timeout -k 10 200 python -u tools/attn_ablate.py --tag abl$v >> gpurun_out/attn_abl.log 2>&1 || exit 1
done
