#!/bin/bash
# CU-mask bit numbering probe, then a kernel trace of the step at --reserve-cus 16 and 32
set -u
O=gpurun_out/cuprobe
mkdir -p $O
timeout -k 10 120 python -u tools/micro/cu_probe.py > $O/probe.log 2>&1 || { echo "probe rc=$?"; tail -20 $O/probe.log; exit 1; }
cat $O/probe.log
cd /tmp && export TMPDIR=/tmp
for r in 16 32; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_r$r -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 3 --reserve-cus $r > $GRAFT_REPO_ROOT/$O/prof_r$r.log 2>&1 || { echo "prof rc=$?"; exit 1; }
done
echo prof ok
