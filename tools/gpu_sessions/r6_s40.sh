#!/bin/bash
# round 6 session 40: last check of the committed HEAD build (after the band switch was removed and
# the extension rebuilt): exchange tests then the bench tests in one process (the order that exposed
# a MASTER_PORT leak from the comm tests into the bench subprocess), the smoke, the driver's command
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s40
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t fused 600 tests/test_comm_gpu.py tests/test_bench_gpu.py
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 $O/smoke.log)"; if crash_rc $rc; then exit 1; fi
b drv 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
echo done
