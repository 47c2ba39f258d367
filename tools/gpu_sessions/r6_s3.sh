#!/bin/bash
# round 6 session 3: HEAD after the pruning of the rejected A/B variants (one-plane conv2 weight
# packs, dy2 LDS row blocks without the unused lo planes, no split / pair / fused-update builds),
# the lazy fc gradient slot and the native store: whole GPU suite + smoke, the driver's command x2
# (peak memory), and a kernel trace of the driver's command.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s3
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t gpu_all 900 tests -m gpu
timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
for i in 1 2; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
echo "peak: $(tail -1 $O/drv_1.log | python3 -c 'import json,sys; c=json.loads(sys.stdin.read())["config"]; print(c["peak_mem_gb"], c.get("store"))')"
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-100)"
# memory-system probes: HBM read / copy / read-modify-write ceilings (the head backward's mix) and the
# texture path's cost per load instruction by address pattern (the conv2 backward's staging)
timeout -k 10 120 tools/micro/rw_bw > $O/rw_bw.log 2>&1 || { echo "rw_bw failed"; tail -5 $O/rw_bw.log; exit 1; }
timeout -k 10 120 tools/micro/ta_pattern > $O/ta_pattern.log 2>&1 || { echo "ta_pattern failed"; tail -5 $O/ta_pattern.log; exit 1; }
cat $O/rw_bw.log $O/ta_pattern.log
echo done
