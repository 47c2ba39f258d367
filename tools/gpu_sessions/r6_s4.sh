#!/bin/bash
# round 6 session 4: the grouped zero-suppressed activation exchange (the head forward in 4
# channel-range launches, each group's rows encoded and gathered right after its launch; the
# deferred update queued group by group before the launch that reads those columns) -- the comm /
# multi-rank GPU tests, the forced exchange at W=1 with and without the 32-CU split and its kernel
# trace, the transport tune, and the OOM demo with the lazy fc gradient slot.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s4
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t comm 600 tests/test_comm_gpu.py tests/test_multirank_gpu.py tests/test_bench_gpu.py -m gpu
b drv 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
for r in 0 32; do
  b fx_$r 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --backend rccl-native --reserve-cus $r --grad-exchange activations
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o fx -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --backend rccl-native --reserve-cus 32 --grad-exchange activations > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-100)"
b tune 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --backend rccl-native --grad-exchange activations --transport-tune
echo "tune: $(tail -1 $O/tune.log | python3 -c 'import json,sys; c=json.loads(sys.stdin.read())["config"]; print(c.get("store"), json.dumps(c["preflight"].get("transport")))')"
timeout -k 10 600 python3 -u tools/oom_demo.py > $O/oom.log 2>&1 || { echo "oom demo rc=$?"; tail -5 $O/oom.log; exit 1; }
echo "oom: $(tail -1 $O/oom.log)"
echo done
