#!/bin/bash
# input prefetch beside the conv2 backward: tests, bench A/B (alternating), kernel trace with prefetch
set -u
O=gpurun_out/prefetch
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_fused_gpu.py \
  tests/test_bench_gpu.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in 1 2 3; do
  for v in no-prefetch prefetch; do
    timeout -k 10 120 python -u bench.py --steps 100 --warmup 10 --$v > $O/bench_${v}_$k.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_${v}_$k.log; exit 1; }
    echo "$v $k: $(tail -1 $O/bench_${v}_$k.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --prefetch > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo prof ok
