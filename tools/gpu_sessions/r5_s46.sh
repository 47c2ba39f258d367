#!/bin/bash
# round 5 session 46: the two latency-bound reductions with more loads in flight -- layer-1
# reduce/finalize 32 / 64 / 128 row lanes per column, conv2 wgrad reduction 4 / 8 / 16 waves
# (base / rf64 / rf128). The driver's command alternating x3, kernel traces of base and rf128,
# then the whole GPU suite on rf128.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s46
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
for i in 1 2 3; do
  for v in base rf64 rf128; do
    V=$v; [ $v = base ] && V=
    b ${v}_$i 200 env TDS_SO_VARIANT=$V python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
for v in base rf128; do
  V=$v; [ $v = base ] && V=
  export TDS_SO_VARIANT=$V
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_$v.log 2>&1 || { echo "prof $v failed"; tail -5 $O/prof_$v.log; exit 1; }
  echo "prof $v: $(grep '^{' $O/prof_$v.log | cut -c1-100)"
done
export TDS_SO_VARIANT=rf128
t gpu_all_rf128 900 tests -m gpu
echo done
