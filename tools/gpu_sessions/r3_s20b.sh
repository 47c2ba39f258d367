#!/bin/bash
# round 3 session 20b: the level-input tests alone (pipeline-shaped levels in the model test), verbose
set -u
O=gpurun_out/r3s20b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -v -s --timeout 200 --timeout-method thread -k "levels or odd_pool" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep -E "ours|FAILED|Error|assert" $O/tests.log | head -40; exit $rc
