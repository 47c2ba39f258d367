#!/bin/bash
# round 4 session 8: forward epilogue (interior fast path, padded staging, no XOR swizzle) and the
# single-workgroup weight pack -- fused tests, then the driver's command alternating with the
# fp16x2 (TDS_CONV2_SPLIT=1) variant build on the same box, and a kernel trace
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/tests.log | head -20; exit 1; }
b() {
  local name=$1; shift
  timeout -k 10 200 env "$@" python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["value"], r["dtype"][:40])')"
}
b tf32_1 TDS_SO_VARIANT=
b split_1 TDS_SO_VARIANT=split
b tf32_2 TDS_SO_VARIANT=
b split_2 TDS_SO_VARIANT=split
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo trace ok
