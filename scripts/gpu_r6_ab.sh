#!/bin/bash
# Paired A/B of library variants on one box: for each round, every variant in VARIANTS ("" = the product library)
# runs `bench.py $BENCH_ARGS`; lines go to gpurun_out/${NAME}_<variant>_<round>.log, the JSON value is printed.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS}; do
    name=${v#+}; [ "$name" = "prod" ] && lib="" || lib=$name
    TAIR_LIB_VARIANT=$lib timeout -k 10 ${LIM:-600} python -u bench.py ${BENCH_ARGS} > gpurun_out/${NAME}_${name}_$r.log 2>&1 || { echo "$name round $r failed"; tail -5 gpurun_out/${NAME}_${name}_$r.log; exit 1; }
    python - "$name" "$r" gpurun_out/${NAME}_${name}_$r.log <<'PY'
import json, sys
for line in open(sys.argv[3]):
    if line.startswith("{"):
        d = json.loads(line)
        print(sys.argv[1], sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["frac"], flush=True)
PY
  done
done
