#!/bin/bash
# rolling conv2 backward: wave-priority variants (timing), then PMC passes over the kernel
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rollprio
mkdir -p $O
for v in "" pm3 ps3; do
  TDS_SO_VARIANT=$v timeout -k 10 90 python -u tools/micro/step_ops_timing.py --iters 30 --only conv2_bwd \
    > $O/t_$v.log 2>&1 || { echo "variant $v rc=$?"; tail -5 $O/t_$v.log; exit 1; }
  echo "variant '$v': $(grep conv2_bwd $O/t_$v.log | head -1)"
done
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex '.*conv2_bwd_roll.*' --output-format csv \
    -d $O/$name -o run -- python3 $R/tools/micro/step_ops_timing.py --only conv2_bwd --iters 2 \
    > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run pa SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 1
run pb SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE || exit 1
run pc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE || exit 1
