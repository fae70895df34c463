#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
run floor2 300 python tools/floor2.py
