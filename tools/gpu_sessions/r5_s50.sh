#!/bin/bash
# round 5 session 50: both reversed consumer walks together (rev2: TDS_F2_REV=1 TDS_L1B_REV=1, p1 stores
# stay non-temporal) against HEAD; r5_s44 had each alone at -6 / -8 us on the driver's command.
# The driver's command alternating x4, kernel traces of both.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s50
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
for i in 1 2 3 4; do
  b head_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  b rev2_$i 200 env TDS_SO_VARIANT=rev2 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
cd /tmp && export TMPDIR=/tmp && cd $R
for v in head rev2; do
  V=$v; [ $v = head ] && V=
  export TDS_SO_VARIANT=$V
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_$v.log 2>&1 || { echo "prof $v failed"; tail -5 $O/prof_$v.log; exit 1; }
  echo "prof $v: $(grep '^{' $O/prof_$v.log | cut -c1-100)"
done
echo done
