#!/bin/bash
# round 3: tiled single-pass zero-suppressed encode (8 pages per workgroup) -- codec + exchange
# tests, forced exchange costs and trace, then the PMC profile of the bench step (r3_pmc.sh)
set -u
O=gpurun_out/r3s7
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_multirank_gpu.py tests/test_comm_gpu.py -v -s \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed" $O/tests.log | tail -12
[ $rc -le 1 ] || { echo "tests rc=$rc"; tail -40 $O/tests.log; exit 1; }
b() {
  local name=$1; shift
  timeout -k 10 200 python -u bench.py "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["config"]["fc_grad"], r["config"]["reserve_cus"], r["config"].get("x_exchange"))')"
}
b bench_1 --steps 30 --warmup 5
b act --steps 30 --warmup 5 --grad-exchange activations
b shd --steps 30 --warmup 5 --grad-exchange sharded
(cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/act_prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --grad-exchange activations > $GRAFT_REPO_ROOT/$O/act_prof.log 2>&1) \
  || { echo "act prof rc=$?"; tail -20 $O/act_prof.log; exit 1; }
echo "act prof ok"
bash tools/gpu_sessions/r3_pmc.sh
