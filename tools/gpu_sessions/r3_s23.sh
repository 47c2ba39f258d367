#!/bin/bash
# round 3 session 23: layer-1 backward with conflict-free LDS (level input: the x tile as bf16 pairs in two
# column-shifted copies, row stride 9 mod 32 banks, one ds_read_b32 per packed B register, no perms;
# dp1 records swizzled so g0/g1 read opposite bank halves) + the hoisted-tap upsample.  Tests, then
# bench x2 (<= 128 VGPRs, 4 WG/CU), the fp32-image bench, kernel trace.
set -u
O=gpurun_out/r3s23
R=$GRAFT_REPO_ROOT
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/bench_def$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_def$i.log; exit 1; }
  echo "default: $(tail -1 $O/bench_def$i.log | cut -c90-200)"
done
timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --input fp32 > $O/bench_fp32.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_fp32.log; exit 1; }
echo "fp32 image: $(tail -1 $O/bench_fp32.log | cut -c90-200)"
(cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 > $R/$O/trace.log 2>&1) || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo "trace ok"
