#!/bin/bash
# round 6 session 18 (timing only): what the head backward's g2m stores cost -- isolated head
# backward with them (default build) and without (_C_nog2m.so, -D TDS_DIAG_NOG2M: wrong results,
# timing only), to size an fp16 g2m
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s18
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
for v in new nog2m new nog2m; do
  if [ $v = new ]; then V=; else V=$v; fi
  OP_ONLY=head_bwd,head_bwd_nomag op hb_$v TDS_SO_VARIANT=$V
done
echo done
