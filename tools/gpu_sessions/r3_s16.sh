#!/bin/bash
# round 3 session 16: conv2 backward knobs re-swept on the no-SLP build (wave priorities of the
# MFMA / staging-load phases, vertical segment length), same box, alternating; then the
# exit-time fault under rocprofv3 with 32 CUs reserved, with the process's library map
set -u
O=gpurun_out/r3s16
mkdir -p $O
for i in 1 2; do
  for v in def p30 p32 p11 s24 s96; do
    vv=$v; [ $v = def ] && vv=
    TDS_SO_VARIANT=$vv timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only conv2_bwd > $O/ops_$v$i.log 2>&1 || { echo "ops rc=$?"; tail -5 $O/ops_$v$i.log; exit 1; }
    echo "$v: $(grep ' ms' $O/ops_$v$i.log | tr '\n' ' ')"
  done
done
R=$GRAFT_REPO_ROOT
(cd /tmp && TMPDIR=/tmp TDS_MAPS_OUT=$R/$O/maps.txt timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/rcus -o run -- \
  python3 $R/tools/micro/exit_maps.py --steps 5 --warmup 2 --reserve-cus 32 > $R/$O/rcus.log 2>&1)
echo "rocprof --reserve-cus 32 rc=$?"
grep -A16 "SIGSEGV" $O/rcus.log | head -20
