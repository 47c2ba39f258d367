#!/bin/bash
# round 6 session 39: the head forward's band (block rows per workgroup) re-measured after the
# one-load-set and fp16-ya changes: 2 / 4 (as built) / 8, by a temporary switch TDS_HEAD_BAND_F;
# head tests at 2 and 8, isolated ops and the driver's command, interleaved
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s39
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
for bnd in 2 8; do
  timeout -k 10 300 env TDS_HEAD_BAND_F=$bnd python -u -m pytest tests/test_fused_gpu.py -k "head" -x -q --timeout 120 --timeout-method thread > $O/kern_$bnd.log 2>&1
  rc=$?; echo "kern band $bnd rc=$rc: $(tail -1 $O/kern_$bnd.log)"; if [ $rc -ne 0 ]; then exit 1; fi
done
for i in 1 2; do
  for bnd in 4 2 8; do
    OP_ONLY=head_fwd,head_bwd op b${bnd}_$i TDS_HEAD_BAND_F=$bnd
  done
done
for i in 1 2; do
  for bnd in 4 8 2; do
    b drv_b${bnd}_$i 200 env TDS_HEAD_BAND_F=$bnd python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  done
done
echo done
