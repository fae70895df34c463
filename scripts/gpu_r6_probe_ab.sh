#!/bin/bash
# Paired A/B of environment settings on the graph-replayed step (tools/graph_launch_probe.py), alternating
# rounds: SETS="A=1,B=0 A=0,B=0" (comma-separated VAR=VALUE lists), BATCH, STEPS, ROUNDS.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
for r in $(seq 1 ${ROUNDS:-2}); do
  for set in ${SETS}; do
    echo "== $set round $r"
    env $(echo $set | tr ',' ' ') timeout -k 10 300 python -u tools/graph_launch_probe.py --batch ${BATCH:-1} --steps ${STEPS:-50} 2>&1 | grep rep || exit 1
  done
done
