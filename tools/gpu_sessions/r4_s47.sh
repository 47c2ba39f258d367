#!/bin/bash
# round 4 session 47: layer-1 launch shapes after the VGPR cuts -- conv workgroups per CU 8 (default)
# vs 4 (variant l1pc4), weight-gradient workgroups per CU 4 (default) vs 5 / 6 (TDS_L1B_PER_CU);
# the driver command x2 each, kernel traces
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s47
mkdir -p $O
cd $R
b() {
  local name=$1; shift
  timeout -k 10 200 env "$@" python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["value"])')"
}
for i in 1 2; do
  b def_$i TDS_SO_VARIANT=
  b pc4_$i TDS_SO_VARIANT=l1pc4
  b lb5_$i TDS_L1B_PER_CU=5
  b lb6_$i TDS_L1B_PER_CU=6
done
cd /tmp && export TMPDIR=/tmp
t() {
  local name=$1; shift
  timeout -k 10 240 env "$@" rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$name -o run -- \
    python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace_$name.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace_$name.log; exit 1; }
}
t def TDS_SO_VARIANT= && t pc4 TDS_SO_VARIANT=l1pc4 && t lb5 TDS_L1B_PER_CU=5 && t lb6 TDS_L1B_PER_CU=6 && echo traces ok
