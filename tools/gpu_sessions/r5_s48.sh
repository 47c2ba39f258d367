#!/bin/bash
# round 5 session 48: finalizer loads clamped instead of guarded (common.h wide_row_sum/max, the conv2
# forward's ypart max, the layer-1 Gram body's sacc/cpg loads, the upsample's source words): the
# compiler had put each guarded load in its own branch and waited for it there. Kernel trace
# (compare with r5_s47 rf128), the driver's command x3, the whole GPU suite + smoke.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s48
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-100)"
for i in 1 2 3; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
t gpu_all 900 tests -m gpu
timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
echo done
