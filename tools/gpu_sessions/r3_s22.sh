#!/bin/bash
# round 3 session 22: upsample with the horizontal taps hoisted out of an 8-row loop (whole 28x28 source in
# LDS); defaults now level input + 4 layer-1 backward workgroups per CU.  Kernel + fused tests, bench x2 (no
# flags = the driver's command), kernel trace
set -u
O=gpurun_out/r3s22
R=$GRAFT_REPO_ROOT
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/bench_$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_$i.log; exit 1; }
  echo "bench: $(tail -1 $O/bench_$i.log | cut -c90-200)"
done
(cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 > $R/$O/trace.log 2>&1) || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo "trace ok"
