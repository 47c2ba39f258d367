#!/bin/bash
# round 6 session 7: HEAD (g2m row-shifted blocks, head backward walking them with plain stores,
# half-item staging) -- the fused kernel tests, then a same-box A/B of the isolated head backward
# and conv2 backward on a real step's tensors and of the driver's command, alternating:
#   HEAD, items (HEAD without the half-item staging: _C_items.so), planar (round-5 g2m and
#   staging: _C_planar.so, the tree of e942132)
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s7
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t fused 400 tests/test_fused_gpu.py tests/test_model_gpu.py -m gpu
for k in 1 2; do
  for v in head items planar; do
    vv=$v; [ $v = head ] && vv=""
    OP_ONLY=head_bwd,conv2_bwd op ${v}_$k TDS_SO_VARIANT=$vv
    b drv_${v}_$k 200 env TDS_SO_VARIANT=$vv python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-100)"
# the transport tune with the probe's buffers freed before each teardown (last: a crash ends the call)
timeout -k 10 200 python3 -X faulthandler -u bench.py --gpus 1 --steps 5 --warmup 2 --backend rccl-native --grad-exchange activations --transport-tune > $O/tune.log 2>&1
echo "tune rc=$?: $(tail -1 $O/tune.log | cut -c1-300)"
echo done
