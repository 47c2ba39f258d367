#!/bin/bash
# round 6 session 5: g2m in the row-shifted pooled-blocked layout (head backward writes 16-B block
# pieces; the conv2 backward's staging loads one block piece + one halo value per lane instead of
# planar row runs) -- the kernel / model / full-scale GPU tests, the driver's command x3 and a
# kernel trace; then the transport tune's crash under faulthandler (its own step, last).
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s5
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t fused 600 tests/test_fused_gpu.py tests/test_fullscale_plan_gpu.py tests/test_model_gpu.py tests/test_bigimage_gpu.py tests/test_comm_gpu.py tests/test_bench_gpu.py -m gpu
timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
for i in 1 2 3; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-100)"
timeout -k 10 200 python3 -X faulthandler -u bench.py --gpus 1 --steps 5 --warmup 2 --backend rccl-native --grad-exchange activations --transport-tune > $O/tune.log 2>&1
echo "tune rc=$?"
grep -A30 "Fatal Python error\|Current thread" $O/tune.log | head -60
echo done
