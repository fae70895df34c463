#!/bin/bash
# Paired A/B of an environment toggle on one box: for each round, every setting in SETTINGS (e.g. "TAIR_EPI_REG=1
# TAIR_EPI_REG=0") runs `bench.py $BENCH_ARGS`; lines go to gpurun_out/${NAME}_<setting>_<round>.log, the JSON value
# is printed.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-2}); do
  for kv in ${SETTINGS}; do
    tag=${kv//=/}
    env "$kv" timeout -k 10 ${LIM:-600} python -u bench.py ${BENCH_ARGS} > gpurun_out/${NAME}_${tag}_$r.log 2>&1 || { echo "$kv round $r failed"; tail -5 gpurun_out/${NAME}_${tag}_$r.log; exit 1; }
    python - "$kv" "$r" gpurun_out/${NAME}_${tag}_$r.log <<'PY'
import json, sys
for line in open(sys.argv[3]):
    if line.startswith("{"):
        d = json.loads(line)
        print(sys.argv[1], sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["frac"], flush=True)
PY
  done
done
