#!/bin/bash
# round 3 session 20c: level-input tests, then the fused + kernel suites, bench A/B levels vs fp32
# image alternating on one box, kernel trace of the levels bench
set -u
O=gpurun_out/r3s20c
R=$GRAFT_REPO_ROOT
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -v --timeout 200 --timeout-method thread -s -k "levels" > $O/tests_lv.log 2>&1
rc=$?; tail -1 $O/tests_lv.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests_lv.log | head -20; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for i in 1 2; do
  for v in levels fp32; do
    timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --input $v > $O/bench_$v$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_$v$i.log; exit 1; }
    echo "$v: $(tail -1 $O/bench_$v$i.log | cut -c90-200)"
  done
done
(cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 > $R/$O/trace.log 2>&1) || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo "trace ok"
