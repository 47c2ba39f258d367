#!/bin/bash
# round 6 session 38: final validation at HEAD (one-load-set head kernels) -- the whole GPU suite
# and the smoke, the driver's command x3, the forced pooled exchange (no split / 32-CU split) and a
# kernel trace of the driver's command
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s38
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t gpu 900 tests -m gpu
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 $O/smoke.log)"; if crash_rc $rc; then exit 1; fi
for i in 1 2 3; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
for r in 0 32; do
  b fx_$r 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --backend rccl-native --reserve-cus $r --grad-exchange activations
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-120)"
echo done
