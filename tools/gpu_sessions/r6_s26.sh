#!/bin/bash
# round 6 session 26: the whole GPU suite and the smoke after ya went to fp16 (r6_s25), plus the
# full-scale numerics printout (-s) of the benchmarked plan for docs/KERNELS.md
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s26
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
timeout -k 10 300 python -u -m pytest tests/test_fullscale_plan_gpu.py tests/test_fullscale_gpu.py -x -q -s --timeout 200 --timeout-method thread > $O/numerics.log 2>&1
rc=$?; echo "numerics rc=$rc: $(tail -1 $O/numerics.log)"; if crash_rc $rc; then exit 1; fi
t gpu 900 tests -m gpu
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 $O/smoke.log)"
echo done
