#!/bin/bash
# round 3 session 17: masked streams released at the end of a --reserve-cus run -- the comm
# tests, the rocprofv3 run that faulted at exit (r3_s14 / r3_s16), smoke, bench x2, then the
# end-of-session kernel trace + 4 PMC passes (r3_pmc_end.sh)
set -u
O=gpurun_out/r3s17
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_comm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
R=$GRAFT_REPO_ROOT
(cd /tmp && TMPDIR=/tmp TDS_MAPS_OUT=$R/$O/maps.txt timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/rcus -o run -- \
  python3 $R/tools/micro/exit_maps.py --steps 5 --warmup 2 --reserve-cus 32 > $R/$O/rcus.log 2>&1)
rc=$?
echo "rocprof --reserve-cus 32 rc=$rc"
[ $rc -eq 0 ] || { grep -A16 "SIGSEGV" $O/rcus.log | head -20; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $O/smoke.log; exit 1; }
echo smoke ok
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > $O/bench_$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench_$i.log; exit 1; }
  echo "bench: $(tail -1 $O/bench_$i.log | cut -c90-190)"
done
timeout -k 10 200 python -u bench.py > $O/bench_default.log 2>&1 || { echo "bench default rc=$?"; tail -20 $O/bench_default.log; exit 1; }
echo "bench (no flags): $(tail -1 $O/bench_default.log | cut -c90-190)"
bash tools/gpu_sessions/r3_pmc_end.sh
