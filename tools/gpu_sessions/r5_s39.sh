#!/bin/bash
# round 5 session 39: end-of-round evidence at HEAD -- python bench.py (100 steps), mnist_onegpu.py
# (100 steps), kernel trace + 4 PMC passes of the step (each pass its own run)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s39
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u bench.py > $O/bench_default.log 2>&1 || { echo "bench rc=$?"; tail -5 $O/bench_default.log; exit 1; }
echo "bench 100: $(tail -1 $O/bench_default.log | cut -c1-200)"
timeout -k 10 300 python3 -u mnist_onegpu.py --epochs 1 --max-steps 100 --json > $O/onegpu.log 2>&1 || { echo "onegpu rc=$?"; tail -5 $O/onegpu.log; exit 1; }
echo "onegpu: $(tail -1 $O/onegpu.log)"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo "trace ok"
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
