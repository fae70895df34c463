#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 900 python bench.py --steps 3 --warmup 1
