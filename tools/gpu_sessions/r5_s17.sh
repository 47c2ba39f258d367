#!/bin/bash
# round 5 session 17: the whole GPU suite (no -x: every failure listed) and smoke() on HEAD
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s17
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_all.log 2>&1
rc=$?
echo "gpu suite rc=$rc: $(tail -1 $O/gpu_all.log)"
grep -E "^(FAILED|ERROR)" $O/gpu_all.log | head -20
case $rc in 124|134|137|139) echo "crash-class exit: stopping"; exit 1 ;; esac
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?: $(tail -1 $O/smoke.log)"
