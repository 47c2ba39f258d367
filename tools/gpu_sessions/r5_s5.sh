#!/bin/bash
# round 5 session 5: the conv2 backward with the wgrad operands 6 steps ahead (default now) --
# staging breakdown in the diag build: 16 full, 17 no staging, 28 staging alone (both MFMA roles
# idle), 60 staging alone without its global loads, 92 staging alone without the BN2/pool math,
# 48 full without staging global loads, 80 full without staging math; GPU tests of conv2 + the
# driver command x2; the exchange's encoder reading ya (test_comm_gpu)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s5
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_model_gpu.py tests/test_comm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
op() {
  local name=$1; shift
  timeout -k 10 240 env "$@" python3 -u tools/micro/step_ops_timing.py --iters 10 --only conv2_bwd > $O/op_$name.log 2>&1 || { echo "op $name rc=$?"; tail -5 $O/op_$name.log; exit 1; }
  echo "op $name: $(grep -v amdgpu.ids $O/op_$name.log | grep -v '^{' | tr '\n' ' ' | cut -c1-300)"
}
op base TDS_SO_VARIANT=
for d in 16 17 28 60 92 48 80; do op d$d TDS_SO_VARIANT=diag TDS_CONV2_DIAG=$d; done
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.log 2>&1 || { echo "drv rc=$?"; tail -5 $O/drv_$i.log; exit 1; }
  echo "drv_$i: $(tail -1 $O/drv_$i.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["value"])')"
done
timeout -k 10 240 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5 > $O/xa32.log 2>&1 || { echo "xa32 rc=$?"; tail -5 $O/xa32.log; exit 1; }
echo "xa32: $(tail -1 $O/xa32.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["value"], r["config"].get("x_exchange"))')"
timeout -k 10 240 python3 -u bench.py --backend rccl-native --reserve-cus 0 --grad-exchange activations --steps 20 --warmup 5 > $O/xa0.log 2>&1 || { echo "xa0 rc=$?"; tail -5 $O/xa0.log; exit 1; }
echo "xa0: $(tail -1 $O/xa0.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["value"])')"
