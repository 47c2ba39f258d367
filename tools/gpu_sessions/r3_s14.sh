#!/bin/bash
# round 3 session 14: -fno-slp-vectorize on the conv kernels (the SLP vectorizer packs f32 math
# into v_pk_* ops, which cost more than scalar ones beside MFMAs) -- same-box A/B against the
# default build (_C_noslp.so, TDS_SO_VARIANT=noslp), alternating; then the round-2 advisor's
# check: one rocprofv3 kernel trace of the bench with 32 CUs reserved (CU-masked streams)
set -u
O=gpurun_out/r3s14
mkdir -p $O
TDS_SO_VARIANT=noslp timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
for i in 1 2; do
  for v in def noslp; do
    vv=$v; [ $v = def ] && vv=
    TDS_SO_VARIANT=$vv timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only l1_fwd,conv2_fwd,conv2_bwd,l1_bwd > $O/ops_$v$i.log 2>&1 || { echo "ops rc=$?"; tail -5 $O/ops_$v$i.log; exit 1; }
    echo "$v: $(grep ' ms' $O/ops_$v$i.log | tr '\n' ' ')"
  done
done
for i in 1 2; do
  for v in def noslp; do
    vv=$v; [ $v = def ] && vv=
    TDS_SO_VARIANT=$vv timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/bench_$v$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_$v$i.log; exit 1; }
    echo "$v: $(tail -1 $O/bench_$v$i.log | cut -c90-190)"
  done
done
R=$GRAFT_REPO_ROOT
(cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/rcus -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 --reserve-cus 32 > $R/$O/rcus.log 2>&1)
echo "rocprof --reserve-cus 32 rc=$?: $(tail -1 $O/rcus.log | cut -c1-200)"
