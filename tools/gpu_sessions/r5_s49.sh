#!/bin/bash
# round 5 session 49: same-box A/B of the clamped finalizer loads (HEAD) against the previous commit's
# build (_C_prev.so: guarded loads, 8564e0f): kernel traces of both, the driver's command alternating x3
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s49
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
cd /tmp && export TMPDIR=/tmp && cd $R
for v in prev head; do
  V=$v; [ $v = head ] && V=
  export TDS_SO_VARIANT=$V
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_$v.log 2>&1 || { echo "prof $v failed"; tail -5 $O/prof_$v.log; exit 1; }
  echo "prof $v: $(grep '^{' $O/prof_$v.log | cut -c1-100)"
done
unset TDS_SO_VARIANT
for i in 1 2 3; do
  b prev_$i 200 env TDS_SO_VARIANT=prev python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  b head_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
echo done
