#!/bin/bash
# round 4 session 36: layer-1 weight gradient x tile as fp16 pair words (one ds_read_b32 per window-row slot pair, no v_perm); tests, then the same-box A/B
# (a worktree of it built in ab_prev/): the driver command alternating x3, a kernel trace of each
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s36
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/tests.log | head -20; exit 1; }
b() {
  local name=$1 dir=$2
  (cd $dir && timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5) > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["value"])')"
}
for i in 1 2 3; do
  b new_$i $R
  b prev_$i $R/ab_prev
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_new -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace_new.log 2>&1 || { echo "trace rc=$?"; exit 1; }
cd $R/ab_prev
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_prev -o run -- \
  python3 $R/ab_prev/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace_prev.log 2>&1 || { echo "trace rc=$?"; exit 1; }
echo traces ok
