#!/bin/bash
# round 6 session 6: the head backward walks g2m's row-shifted blocks (its 4 waves write one block's
# 4 rows in one iteration, plain stores): the fused kernel tests, the driver's command x2 and a trace
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s6
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t fused 400 tests/test_fused_gpu.py tests/test_model_gpu.py -m gpu
for i in 1 2; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-100)"
echo done
