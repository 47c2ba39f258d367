#!/bin/bash
# round 4 session 44: head backward band 2 block rows (its own grid; forward stays 4) -- fused/model tests,
# then the driver
# command alternating with the band-4 backward (TDS_HP_BAND_B=4, variant bb4), kernel traces
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s44
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/tests.log | head -20; exit 1; }
b() {
  local name=$1; shift
  timeout -k 10 200 env "$@" python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["value"])')"
}
for i in 1 2 3; do
  b new_$i TDS_SO_VARIANT=
  b bb4_$i TDS_SO_VARIANT=bb4
done
cd /tmp && export TMPDIR=/tmp
for v in new bb4; do
  sv=$v; [ $v = new ] && sv=
  timeout -k 10 240 env TDS_SO_VARIANT=$sv rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace_$v.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace_$v.log; exit 1; }
  echo "trace $v ok"
done
