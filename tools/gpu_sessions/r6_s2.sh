#!/bin/bash
# round 6 session 2: the fc gradient slot no longer requested by the fused head backward (lazy slot
# never allocated), CE label guard, native store default; the driver's command x2 (peak memory),
# the OOM demo at the new edge, the forced exchange at reserve 0 / 32 / 64 (split costs of
# parallel/transport_tune.py) and the transport tune itself at W=1
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s2
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t sel 600 tests/test_fullscale_plan_gpu.py tests/test_kernels_gpu.py tests/test_comm_gpu.py tests/test_bench_gpu.py tests/test_model_gpu.py tests/test_head_ce_gpu.py -m gpu
for i in 1 2; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
echo "peak: $(tail -1 $O/drv_1.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["config"]["peak_mem_gb"])')"
for r in 0 32 64; do
  b fx_$r 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --backend rccl-native --reserve-cus $r --grad-exchange activations
done
b tune 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --backend rccl-native --grad-exchange activations --transport-tune
echo "tune: $(tail -1 $O/tune.log | python3 -c 'import json,sys; c=json.loads(sys.stdin.read())["config"]; print(c.get("store"), json.dumps(c["preflight"].get("transport")))')"
timeout -k 10 600 python3 -u tools/oom_demo.py > $O/oom.log 2>&1 || { echo "oom demo rc=$?"; tail -5 $O/oom.log; exit 1; }
echo "oom: $(tail -1 $O/oom.log)"
echo done
