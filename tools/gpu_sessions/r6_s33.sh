#!/bin/bash
# round 6 session 33: the pooled update (head_upd_pb_kernel) with every rank's images of a pass loaded
# together (NR 1 / 2 / 4) against one rank at a time (TDS_UPD_NR=1, a temporary switch), isolated at
# the bench shape for 1, 2, 4 and 8 source ranks; the kernel test first
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s33
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
# (kernel test: passed in the first run of this script)
for i in 1 2; do
  timeout -k 10 200 env TDS_UPD_NR=1 python3 -u tools/micro/pooled_update_timing.py --ranks 1,2,4,8 > $O/nr1_$i.log 2>&1 || { echo "nr1 failed"; tail -5 $O/nr1_$i.log; exit 1; }
  echo "nr1_$i: $(grep ranks $O/nr1_$i.log | tr '\n' ' ')"
  timeout -k 10 200 python3 -u tools/micro/pooled_update_timing.py --ranks 1,2,4,8 > $O/nrx_$i.log 2>&1 || { echo "nrx failed"; tail -5 $O/nrx_$i.log; exit 1; }
  echo "nrx_$i: $(grep ranks $O/nrx_$i.log | tr '\n' ' ')"
done
echo done
