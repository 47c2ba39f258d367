#!/bin/bash
# round 3 session 23: opt-in layer-1 backward pair layout (TDS_L1B_PAIRS=1: conflict-free bf16-pair x tile,
# swizzled dp1 records; 144 VGPRs -> 3 WG/CU) and whole-source upsample (TDS_UPS_IMG=1, hoisted taps):
# tests on both settings, then bench A/B alternating against the default, kernel traces
set -u
O=gpurun_out/r3s23
R=$GRAFT_REPO_ROOT
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
TDS_L1B_PAIRS=1 TDS_L1B_PER_CU=3 TDS_UPS_IMG=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -q --timeout 200 --timeout-method thread -k "upsample or layer1 or levels" > $O/tests_opt.log 2>&1
rc=$?; tail -1 $O/tests_opt.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests_opt.log | head -20; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/bench_def$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_def$i.log; exit 1; }
  echo "default: $(tail -1 $O/bench_def$i.log | cut -c90-200)"
  TDS_L1B_PAIRS=1 TDS_L1B_PER_CU=3 timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/bench_pairs$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_pairs$i.log; exit 1; }
  echo "pairs: $(tail -1 $O/bench_pairs$i.log | cut -c90-200)"
  TDS_UPS_IMG=1 timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/bench_img$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_img$i.log; exit 1; }
  echo "ups img: $(tail -1 $O/bench_img$i.log | cut -c90-200)"
done
(cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 > $R/$O/trace.log 2>&1) || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
(cd /tmp && TMPDIR=/tmp TDS_L1B_PAIRS=1 TDS_L1B_PER_CU=3 TDS_UPS_IMG=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace_opt -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 > $R/$O/trace_opt.log 2>&1) || { echo "trace opt rc=$?"; tail -5 $O/trace_opt.log; exit 1; }
echo "trace ok"
