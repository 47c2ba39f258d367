#!/bin/bash
# round 3 session 11: same-box A/B of the tile-table layout (TDS_TILE_LISTS=0: work-index-major,
# 1: per-workgroup lists), alternating, conv2 fwd/bwd op timings and the bench
set -u
O=gpurun_out/r3s11
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
for i in 1 2; do
  for v in 0 1; do
    TDS_TILE_LISTS=$v timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only conv2_fwd,conv2_bwd,head_bwd > $O/ops_$v$i.log 2>&1 || { echo "ops rc=$?"; tail -5 $O/ops_$v$i.log; exit 1; }
    echo "lists=$v: $(grep ' ms' $O/ops_$v$i.log | tr '\n' ' ')"
  done
done
for i in 1 2; do
  for v in 0 1; do
    TDS_TILE_LISTS=$v timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/bench_$v$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_$v$i.log; exit 1; }
    echo "lists=$v: $(tail -1 $O/bench_$v$i.log | cut -c90-190)"
  done
done
