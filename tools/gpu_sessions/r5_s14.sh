#!/bin/bash
# round 5 session 14: PMC of the isolated conv2 backward (step_ops_timing --only conv2_bwd), one
# counter group per pass: the texture address / data path and L1 stalls (is the staging role's
# load path the limiter?), L2 hit / miss, and the wave's instruction mix
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r5s14
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
# the whole GPU suite and smoke() first, as the driver runs them at round end
t gpu_all 900 tests -m gpu
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?: $(tail -1 $O/smoke.log)"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1 ctr=$2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $O/$name -o run -- \
    python3 $R/tools/micro/step_ops_timing.py --iters 3 --only conv2_bwd > $O/$name.log 2>&1
  echo "$name rc=$?"
}
run pa "GRBM_GUI_ACTIVE TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum"
run pb "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
run pc "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
run pd "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"
run pe "SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_SALU"
