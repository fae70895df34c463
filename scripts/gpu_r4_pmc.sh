#!/bin/bash
# Round-4 rocprof evidence: kernel stats + PMC summaries for configs[1] (B=1), configs[2] micro-batch (B=64), fp8 B=1.
set -o pipefail
B=1 TAG=r04b1 bash scripts/gpu_profile.sh || exit 1
B=64 TAG=r04b64 bash scripts/gpu_profile.sh || exit 1
B=1 FP8=1 TAG=r04b1_fp8 bash scripts/gpu_profile.sh || exit 1
