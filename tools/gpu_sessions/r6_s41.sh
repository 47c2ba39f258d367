#!/bin/bash
# round 6 session 41: the head backward's band (block rows per workgroup) 2 (as built) vs 4 after the
# one-load-set and fp16-ya changes, by a temporary switch TDS_HEAD_BAND_B; the fused tests at 4, then
# isolated ops and the driver's command, interleaved
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s41
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
timeout -k 10 300 env TDS_HEAD_BAND_B=4 python -u -m pytest tests/test_fused_gpu.py tests/test_bigimage_gpu.py -x -q --timeout 120 --timeout-method thread > $O/kern4.log 2>&1
rc=$?; echo "kern band 4 rc=$rc: $(tail -1 $O/kern4.log)"; if [ $rc -ne 0 ]; then exit 1; fi
for i in 1 2; do
  for bnd in 2 4; do
    OP_ONLY=head_bwd op b${bnd}_$i TDS_HEAD_BAND_B=$bnd
  done
done
for i in 1 2 3; do
  for bnd in 2 4; do
    b drv_b${bnd}_$i 200 env TDS_HEAD_BAND_B=$bnd python3 -u bench.py --gpus 1 --steps 20 --warmup 5
  done
done
echo done
