#!/bin/bash
# PMC passes over the conv2 backward kernel (one counter group per run)
set -u
mkdir -p gpurun_out/pmc_b3
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex '.*conv2_bwd3.*' --output-format csv \
    -d $R/gpurun_out/pmc_b3/$name -o run -- python3 $R/tools/micro/step_ops_timing.py --only conv2_bwd --iters 2 \
    > $R/gpurun_out/pmc_b3/$name.log 2>&1
  echo "$name rc=$?"
}
run p1 TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum || exit 1
run p2 TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE || exit 1
run p3 TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_STALL_MULTI_MISS_sum SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE || exit 1
