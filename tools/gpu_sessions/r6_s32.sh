#!/bin/bash
# round 6 session 32: the whole GPU suite and the smoke at HEAD (r6_s31 stopped at the bench
# preflight test, whose expectation predated the pooled exchange)
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s32
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t gpu 900 tests -m gpu
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 $O/smoke.log)"
echo done
