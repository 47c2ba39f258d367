#!/bin/bash
# round 4 session 43: head kernels' band height (block rows per workgroup) 4 (default) vs 2 vs 8,
# re-swept after the reverse-order head backward -- the driver command alternating x2, traces
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s43
mkdir -p $O
cd $R
b() {
  local name=$1; shift
  timeout -k 10 200 env "$@" python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["value"])')"
}
for i in 1 2; do
  b b4_$i TDS_SO_VARIANT=
  b b2_$i TDS_SO_VARIANT=hb2
  b b8_$i TDS_SO_VARIANT=hb8
done
cd /tmp && export TMPDIR=/tmp
for v in b4 hb2 hb8; do
  sv=$v; [ $v = b4 ] && sv=
  timeout -k 10 240 env TDS_SO_VARIANT=$sv rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace_$v.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace_$v.log; exit 1; }
  echo "trace $v ok"
done
