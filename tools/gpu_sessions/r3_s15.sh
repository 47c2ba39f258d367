#!/bin/bash
# round 3 session 15: conv2 kernels built without SLP vectorization (default now) -- full GPU
# suite; bitwise check of the fma_mix fp16 split; same-box A/B of (a) the head / exchange
# kernels without SLP (_C_noslp2.so) and (b) the staging's fp16 split by v_fma_mix (_C_mix.so);
# then the exit-time fault under rocprofv3 with 32 CUs reserved, with the process's library map
set -u
O=gpurun_out/r3s15
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
timeout -k 10 60 ./tools/micro/f16_split_check > $O/split.log 2>&1 || { echo "split check rc=$?"; cat $O/split.log; exit 1; }
cat $O/split.log
TDS_SO_VARIANT=mix timeout -k 10 300 python -u -m pytest tests/test_fused_gpu.py tests/test_fullscale_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests_mix.log 2>&1
rc=$?; tail -1 $O/tests_mix.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests_mix.log | head; exit 1; }
for i in 1 2; do
  for v in def noslp2 mix; do
    vv=$v; [ $v = def ] && vv=
    TDS_SO_VARIANT=$vv timeout -k 10 120 python -u tools/micro/step_ops_timing.py --iters 20 --only head_fwd,head_bwd,conv2_bwd > $O/ops_$v$i.log 2>&1 || { echo "ops rc=$?"; tail -5 $O/ops_$v$i.log; exit 1; }
    echo "$v: $(grep ' ms' $O/ops_$v$i.log | tr '\n' ' ')"
  done
done
for i in 1 2; do
  for v in def noslp2 mix; do
    vv=$v; [ $v = def ] && vv=
    TDS_SO_VARIANT=$vv timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/bench_$v$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_$v$i.log; exit 1; }
    echo "$v: $(tail -1 $O/bench_$v$i.log | cut -c90-190)"
  done
done
R=$GRAFT_REPO_ROOT
(cd /tmp && TMPDIR=/tmp TDS_MAPS_OUT=$R/$O/maps.txt timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/rcus -o run -- \
  python3 $R/tools/micro/exit_maps.py --steps 5 --warmup 2 --reserve-cus 32 > $R/$O/rcus.log 2>&1)
echo "rocprof --reserve-cus 32 rc=$?"
grep -A16 "SIGSEGV" $O/rcus.log | head -20
