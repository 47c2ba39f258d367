#!/bin/bash
# round 5 session 35: rows per wave of the fused upsample + moments (TDS_UM_RB 32 / 40 / 48 / 64),
# isolated op (median of 5 x 20 calls), alternating
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s35
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
for r in 1 2; do
  OP_ONLY=ups_mom op rb48_$r TDS_SO_VARIANT=
  OP_ONLY=ups_mom op rb32_$r TDS_SO_VARIANT=rb32
  OP_ONLY=ups_mom op rb40_$r TDS_SO_VARIANT=rb40
  OP_ONLY=ups_mom op rb64_$r TDS_SO_VARIANT=rb64
done

# the layer-1 backward's reducer with its inputs staged before the hand-off
t tests 600 tests/test_fused_gpu.py tests/test_fullscale_plan_gpu.py
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/l1b -o run -- python3 -u tools/micro/step_ops_timing.py --iters 10 --only l1_bwd > $O/l1b.log 2>&1 || { echo "l1b failed"; tail -5 $O/l1b.log; exit 1; }
echo "l1b: $(grep -h 'reduce_finalize' $O/l1b/run_kernel_stats.csv | cut -d, -f1-6 | cut -c1-200)"
echo done2
