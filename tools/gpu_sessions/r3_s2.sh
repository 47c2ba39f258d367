#!/bin/bash
# round 3: fp16x2 conv2 + zero-suppressed exchange -- fused numerics first, then the full GPU
# suite, smoke, driver-shaped bench x2, W=1 forced-exchange costs, fc-input sparsity, kernel trace
set -u
O=gpurun_out/r3s2
mkdir -p $O
# test failures (rc 1) do not stop the session; a crash, abort or time limit does
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed" $O/tests.log | tail -12
[ $rc -le 1 ] || { echo "tests rc=$rc"; tail -40 $O/tests.log; exit 1; }
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
b() {
  local name=$1; shift
  timeout -k 10 200 python -u bench.py "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | cut -c1-200)"
}
b bench_1 --steps 20 --warmup 5
b bench_2 --steps 20 --warmup 5
b bench_100 --steps 100 --warmup 10
b act_zs --steps 20 --warmup 5 --grad-exchange activations
b act_dense --steps 20 --warmup 5 --grad-exchange activations --no-exchange-compress
b sharded --steps 20 --warmup 5 --grad-exchange sharded
timeout -k 10 300 python -u tools/x_sparsity.py > $O/xsp.log 2>&1 || { echo "xsp rc=$?"; tail -20 $O/xsp.log; exit 1; }
tail -1 $O/xsp.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo prof ok
