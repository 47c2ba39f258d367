#!/bin/bash
# round 5 session 44: Infinity Cache reuse of the step's 360 MB producer -> consumer tensors.
# rev: the conv2 forward walks p1 last-to-first (the layer-1 conv writes it first-to-last);
# revpl: rev + plain (allocating) p1 stores instead of non-temporal; l1brev: the layer-1 backward
# walks dp1 last-to-first (the conv2 backward writes it first-to-last); all3: all of them.
# The driver's command alternating x3, then a kernel trace of each arm.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s44
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
for i in 1 2 3; do
  for v in base rev revpl l1brev all3; do
    V=$v; [ $v = base ] && V=
    b ${v}_$i 200 env TDS_SO_VARIANT=$V python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
for v in base revpl l1brev all3; do
  V=$v; [ $v = base ] && V=
  export TDS_SO_VARIANT=$V
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_$v.log 2>&1 || { echo "prof $v failed"; tail -5 $O/prof_$v.log; exit 1; }
  echo "prof $v: $(grep '^{' $O/prof_$v.log | cut -c1-100)"
done
echo done
