#!/bin/bash
# round 4 session 28: head backward workgroups in the reverse of the forward's order (MALL reuse of
# the forward's last-streamed ya / weight lines) -- fused/model tests, then the driver's command
# alternating with the forward-order variant build (rev0) on the same box, and a kernel trace of each
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s28
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/tests.log | head -20; exit 1; }
b() {
  local name=$1; shift
  timeout -k 10 200 env "$@" python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["value"])')"
}
for i in 1 2 3; do
  b rev_$i TDS_SO_VARIANT=
  b fwd_$i TDS_SO_VARIANT=rev0
done
cd /tmp && export TMPDIR=/tmp
for v in "" rev0; do
  timeout -k 10 240 env TDS_SO_VARIANT=$v rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_${v:-rev} -o run -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace_${v:-rev}.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace_${v:-rev}.log; exit 1; }
  echo "trace ${v:-rev} ok"
done
