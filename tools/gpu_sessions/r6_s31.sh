#!/bin/bash
# round 6 session 31: end-of-round evidence at HEAD (fp16 g2m and ya, pooled exchange) -- the whole
# GPU suite and the smoke, the driver's command x3, the forced pooled exchange (no split / 32-CU
# split), a kernel trace of the driver's command, 4 PMC passes
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s31
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
run() {
  local name=$1; shift
  timeout -s KILL 200 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run pa SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE || exit 1
run pb TCC_EA0_RDREQ_DRAM_32B_sum GRBM_GUI_ACTIVE || exit 1
run pc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE || exit 1
run pd SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE || exit 1
echo done
