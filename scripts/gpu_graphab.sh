#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
run graphab_single 300 env TAIR_CN_FORK=0 TAIR_ZC_OVERLAP=0 python tools/graph_ab.py
run graphab_fork 300 python tools/graph_ab.py
