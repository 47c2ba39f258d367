#!/bin/bash
# validation after the launch-shape changes: full GPU suite, smoke, bench x2, 32-row autocorrelation variant, kernel trace
set -u
O=gpurun_out/val3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
b() {
  local name=$1; shift
  timeout -k 10 150 python -u bench.py "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
}
for v in "" ac32; do
  TDS_SO_VARIANT=$v timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 > $O/t_$v.log 2>&1 || { echo "ops $v rc=$?"; tail -5 $O/t_$v.log; exit 1; }
  echo "ops '$v': $(tail -1 $O/t_$v.log)"
done
TDS_SO_VARIANT=ac32 timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_fused_gpu.py -k layer1 > $O/tests_ac32.log 2>&1 || { echo "ac32 tests rc=$?"; tail -20 $O/tests_ac32.log; exit 1; }
for k in 1 2; do
  b def_$k
  TDS_SO_VARIANT=ac32 b ac32_$k
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo prof ok
