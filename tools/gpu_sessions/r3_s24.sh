#!/bin/bash
# round 3 session 24: final validation of the defaults (uint8 level input, whole-source upsample, layer-1
# backward 4 WG/CU): full GPU suite, smoke, bench x2 with no flags (the driver's command), kernel trace
set -u
O=gpurun_out/r3s24
R=$GRAFT_REPO_ROOT
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -1 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head; exit 1; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
echo smoke ok
for i in 1 2; do
  timeout -k 10 200 python -u bench.py > $O/bench_$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_$i.log; exit 1; }
  echo "bench: $(tail -1 $O/bench_$i.log | cut -c90-200)"
done
(cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 > $R/$O/trace.log 2>&1) || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo "trace ok"
