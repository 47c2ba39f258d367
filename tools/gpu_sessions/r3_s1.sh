#!/bin/bash
# round 3, first session: full GPU suite (incl. the new toy/OOM-rehearsal/layers-exchange tests),
# smoke, driver-shaped bench x2, fc-input sparsity at the bench shape, kernel trace of the bench
set -u
O=gpurun_out/r3s1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for k in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 > $O/bench_$k.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_$k.log; exit 1; }
  tail -1 $O/bench_$k.log | cut -c1-220
done
timeout -k 10 300 python -u tools/x_sparsity.py > $O/xsp.log 2>&1 || { echo "xsp rc=$?"; tail -20 $O/xsp.log; exit 1; }
tail -1 $O/xsp.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo prof ok
