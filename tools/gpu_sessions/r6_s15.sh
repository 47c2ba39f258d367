#!/bin/bash
# round 6 session 15: HEAD validation after the conv2 / layer-1 epilogue work -- whole GPU suite +
# smoke, the driver's command x3, the forced exchange (32-CU split), a kernel trace of the driver's
# command and 4 PMC passes of the step (the end-of-round evidence for docs/KERNELS.md)
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s15
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t gpu_all 900 tests -m gpu
timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
for i in 1 2 3; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
echo "peak: $(tail -1 $O/drv_1.log | python3 -c 'import json,sys; c=json.loads(sys.stdin.read())["config"]; print(c["peak_mem_gb"], c.get("store"))')"
b fx_32 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --backend rccl-native --reserve-cus 32 --grad-exchange activations
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
