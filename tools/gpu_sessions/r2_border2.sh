#!/bin/bash
# per-image border strip workgroups: full GPU suite, op timing, bench
set -u
O=gpurun_out/border2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 > $O/ops.log 2>&1 || { echo "ops rc=$?"; tail -5 $O/ops.log; exit 1; }
tail -1 $O/ops.log
for k in 1 2; do
  timeout -k 10 150 python -u bench.py > $O/bench_$k.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_$k.log; exit 1; }
  tail -1 $O/bench_$k.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])'
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo prof ok
