#!/bin/bash
# round 4 session 1: baseline on this round's box -- the driver's exact command x3 vs the 100-step default x2,
# then a kernel trace of the driver command (per-step variance after a 5-step warmup)
set -u
O=gpurun_out/r4s1
R=$GRAFT_REPO_ROOT
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/drv_$i.log; exit 1; }
  echo "drv: $(tail -1 $O/drv_$i.log | cut -c90-200)"
done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py > $O/def_$i.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/def_$i.log; exit 1; }
  echo "def: $(tail -1 $O/def_$i.log | cut -c90-200)"
done
(cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 > $R/$O/trace.log 2>&1) || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo "trace ok"
