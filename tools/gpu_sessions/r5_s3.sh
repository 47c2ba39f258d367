#!/bin/bash
# round 5 session 3: the in-launch finalizers with write-through hand-off stores (no per-workgroup
# release fence) under the fused / model / determinism GPU tests + smoke; driver command A/B
# against the separate finalize launches (TDS_FUSED_FIN=0); the full-scale two-step plan test;
# kernel traces of the local and the forced-exchange step
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s3
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_model_gpu.py tests/test_determinism_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
b() {
  local name=$1; shift
  timeout -k 10 200 env "$@" python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["value"])')"
}
for i in 1 2; do
  b fin_$i TDS_FUSED_FIN=1
  b sep_$i TDS_FUSED_FIN=0
done
timeout -k 10 900 python -u -m pytest tests/test_fullscale_plan_gpu.py -x -v -s --timeout 900 --timeout-method thread > $O/plan_test.log 2>&1 || { echo "plan test rc=$?"; grep -A40 "benchmarked plan" $O/plan_test.log | head -50; exit 1; }
grep -A40 "benchmarked plan" $O/plan_test.log | head -45
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_loc -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace_loc.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace_loc.log; exit 1; }
echo "trace_loc ok"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_xa -o run -- \
  python3 $R/bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5 > $O/trace_xa.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace_xa.log; exit 1; }
echo "trace_xa ok"
