#!/bin/bash
source "$(dirname "$0")/gpu_tests.sh"
run launch_floor 300 python tools/launch_floor.py
run kernel_floor 300 python tools/kernel_floor.py
