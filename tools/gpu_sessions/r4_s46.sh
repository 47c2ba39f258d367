#!/bin/bash
# round 4 session 46: head band heights around the defaults (forward 4, backward 2): forward 3 / 5 / 6,
# backward 1 / 3 -- the driver command x2 each, kernel traces
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s46
mkdir -p $O
cd $R
b() {
  local name=$1; shift
  timeout -k 10 200 env "$@" python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["value"])')"
}
for i in 1 2; do
  for v in def f3 f5 f6 b1 b3; do
    sv=$v; [ $v = def ] && sv=
    b ${v}_$i TDS_SO_VARIANT=$sv
  done
done
cd /tmp && export TMPDIR=/tmp
for v in def f3 f5 f6 b1 b3; do
  sv=$v; [ $v = def ] && sv=
  timeout -k 10 240 env TDS_SO_VARIANT=$sv rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace_$v.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace_$v.log; exit 1; }
done
echo traces ok
