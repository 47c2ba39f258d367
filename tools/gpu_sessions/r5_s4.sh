#!/bin/bash
# round 5 session 4: (1) one-round ("wide") reducers in the in-launch finalizers: fused / model GPU
# tests + smoke, driver-command A/B against the separate launches (TDS_FUSED_FIN=0); (2) conv2
# backward operand prefetch depth: wgrad B operands 4 / 6 steps ahead (flat ring, variants wg4,
# wg6), dgrad A rows 4 ahead (wg6d4) -- isolated op and driver command; (3) role clocks of the
# deeper-prefetch diag build (dwg6d4: 16 full, 17 no staging, 21 wgrad only, 25 dgrad only);
# (4) trace of the forced-exchange step (teardown fixed)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s4
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
b() {
  local name=$1; shift
  timeout -k 10 200 env "$@" python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["value"])')"
}
op() {
  local name=$1; shift
  timeout -k 10 240 env "$@" python3 -u tools/micro/step_ops_timing.py --iters 10 --only conv2_bwd > $O/op_$name.log 2>&1 || { echo "op $name rc=$?"; tail -5 $O/op_$name.log; exit 1; }
  echo "op $name: $(grep -v amdgpu.ids $O/op_$name.log | grep -v '^{' | tr '\n' ' ' | cut -c1-300)"
}
for v in base wg4 wg6 wg6d4; do
  sv=$v; [ $v = base ] && sv=
  op $v TDS_SO_VARIANT=$sv
done
for d in 16 17 21 25; do op dwg6d4_$d TDS_SO_VARIANT=dwg6d4 TDS_CONV2_DIAG=$d; done
for i in 1 2; do
  b fin_$i TDS_FUSED_FIN=1
  b sep_$i TDS_FUSED_FIN=0
  b wg6_$i TDS_SO_VARIANT=wg6
  b wg6d4_$i TDS_SO_VARIANT=wg6d4
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_loc -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace_loc.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace_loc.log; exit 1; }
echo "trace_loc ok"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_xa -o run -- \
  python3 $R/bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5 > $O/trace_xa.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace_xa.log; exit 1; }
echo "trace_xa ok"
