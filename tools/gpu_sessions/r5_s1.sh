#!/bin/bash
# round 5 session 1: HEAD baseline on this round's box -- the driver's command, the forced
# activation exchange at W=1 (rccl-native, 32-CU split and without it, no-exchange split cost),
# the conv2/model GPU tests after the per-tile fp64 BN2 partials, and kernel traces of the local step and the forced-exchange step
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s1
mkdir -p $O
cd $R
run() {  # name timeout args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python3 -u bench.py "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?"; tail -20 $O/$n.log; exit 1; }
  echo "$n: $(tail -1 $O/$n.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); c=r["config"]; print(r["ms_per_step"], r["value"], c.get("fc_grad"), c.get("reserve_cus"), c.get("x_exchange",""))')"
}
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
run drv 200 --gpus 1 --steps 20 --warmup 5
run xa32 240 --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
run xa0 240 --backend rccl-native --reserve-cus 0 --grad-exchange activations --steps 20 --warmup 5
run loc32 240 --backend rccl-native --reserve-cus 32 --steps 20 --warmup 5
run drv2 200 --gpus 1 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_loc -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace_loc.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace_loc.log; exit 1; }
echo "trace_loc ok"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_xa -o run -- \
  python3 $R/bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5 > $O/trace_xa.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace_xa.log; exit 1; }
echo "trace_xa ok"
cd $R
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
timeout -k 10 900 python -u -m pytest tests/test_fullscale_plan_gpu.py -x -v -s --timeout 900 --timeout-method thread > $O/plan_test.log 2>&1 || { echo "plan test rc=$?"; tail -40 $O/plan_test.log; exit 1; }
grep -A40 "benchmarked plan" $O/plan_test.log | head -60
