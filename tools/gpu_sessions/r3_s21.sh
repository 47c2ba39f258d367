#!/bin/bash
# round 3 session 21: layer-1 backward held to <= 128 VGPRs (__launch_bounds__(256, 3); the level variant
# had grown to 176 VGPRs = 2 waves per SIMD and ran 0.56 ms); bench A/B of input levels / fp32 image x
# layer-1 backward workgroups per CU 3 / 4, alternating on one box; kernel trace of the levels bench;
# upsample: whole 28x28 source staged, 8 output rows per workgroup
set -u
O=gpurun_out/r3s21
R=$GRAFT_REPO_ROOT
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit 1; }
for i in 1 2; do
  for wg in 3 4; do
    for v in levels fp32; do
      TDS_L1B_PER_CU=$wg timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --input $v > $O/bench_$v${wg}_$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_$v${wg}_$i.log; exit 1; }
      echo "$v wg$wg: $(tail -1 $O/bench_$v${wg}_$i.log | cut -c90-200)"
    done
  done
done
(cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 --input levels > $R/$O/trace.log 2>&1) || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
(cd /tmp && TMPDIR=/tmp TDS_L1B_PER_CU=4 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace4 -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 --input levels > $R/$O/trace4.log 2>&1) || { echo "trace4 rc=$?"; tail -5 $O/trace4.log; exit 1; }
echo "trace ok"
