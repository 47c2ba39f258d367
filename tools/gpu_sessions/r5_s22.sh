#!/bin/bash
# round 5 session 22: the input op and the x moments in isolation (levels input), with and without
# the border-strip workgroups (TDS_AC_BORDER=0: A/B timing only)
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s22
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
OP_ONLY=ups,moments,l1_fwd op base TDS_AC_BORDER=1
OP_ONLY=moments op noborder TDS_AC_BORDER=0
OP_ONLY=ups,moments op base2 TDS_AC_BORDER=1
echo done
