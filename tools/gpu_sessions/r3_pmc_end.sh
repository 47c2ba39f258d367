#!/bin/bash
# round 3 end-of-session profile (no-SLP conv2) of the bench step: kernel trace + 4 PMC passes (counter limits per
# block respected: <= 8 SQ, <= 4 TCC).  HBM read bytes from the per-size DRAM request counter
# (TCC_EA0_RDREQ_DRAM_32B: 32-B units, a 64-B request counts 2, a 128-B one 4), which matches
# tensor sizes, unlike FETCH_SIZE (half of a wide streaming read on gfx950).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3pmc_end
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --steps 10 --warmup 3 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo "trace ok: $(tail -1 $O/trace.log | cut -c1-160)"
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
echo pmc ok
