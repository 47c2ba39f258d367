#!/bin/bash
# round 5 session 2: where the conv2 backward's MFMA waves lose their time -- timing-only flag
# variants of the diag build (conv2_common.h: 16 = full + clocks; +1 no staging, +2 no LDS operand
# reads in the MFMA waves, +4 dgrad idle, +8 wgrad idle), each with per-role barrier clocks, the
# isolated op on a real step's tensors (tools/micro/step_ops_timing.py)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s2
mkdir -p $O
cd $R
for d in 0 16 17 19 21 25 23 27 20 24; do
  timeout -k 10 240 env TDS_SO_VARIANT=diag TDS_CONV2_DIAG=$d python3 -u tools/micro/step_ops_timing.py --iters 10 \
    --only conv2_bwd > $O/diag_$d.log 2>&1 || { echo "diag $d rc=$?"; tail -5 $O/diag_$d.log; exit 1; }
  echo "diag $d: $(grep -v amdgpu.ids $O/diag_$d.log | grep -v '^{' | tr '\n' ' ' | cut -c1-400)"
done
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
timeout -k 10 900 python -u -m pytest tests/test_fullscale_plan_gpu.py -x -v -s --timeout 900 --timeout-method thread > $O/plan_test.log 2>&1 || { echo "plan test rc=$?"; tail -40 $O/plan_test.log; exit 1; }
grep -A40 "benchmarked plan" $O/plan_test.log | head -60
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_xa -o run -- \
  python3 $R/bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5 > $O/trace_xa.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace_xa.log; exit 1; }
echo "trace_xa ok"
