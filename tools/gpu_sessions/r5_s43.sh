#!/bin/bash
# round 5 session 43: final HEAD validation; whole GPU suite + smoke, the driver's command x3, the forced
# activation exchange at W = 1 (rccl-native, 32-CU split) and the same split without the exchange,
# kernel trace of the driver's command
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s43
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t gpu_all 900 tests -m gpu
timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
for i in 1 2 3; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
for i in 1 2; do
  b xa_$i 240 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
  b loc32_$i 240 python3 -u bench.py --backend rccl-native --reserve-cus 32 --steps 20 --warmup 5
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-120)"
echo done
