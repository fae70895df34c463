#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
run gemmcmp 300 python tools/gemm_vs_blas.py
