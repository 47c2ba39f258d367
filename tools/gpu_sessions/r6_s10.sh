#!/bin/bash
# round 6 session 10: the copy-only clock warm-up (per-step times) and a 25-step warmup for the
# steady state; kernel traces of the driver's command and of the forced exchange (1 and 4 groups);
# 4 PMC passes of the step; then the OOM demo with the constructor / step peaks modelled apart
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s10
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
for i in 1 2; do
  b cwc_$i 200 env TDS_CLOCK_WARMUP=copy python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --step-times --clock-warmup-ms 1000
  echo "  steps: $(tail -1 $O/cwc_$i.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["config"]["step_ms"])')"
done
b w25 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 25 --step-times
echo "  steps: $(tail -1 $O/w25.log | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["config"]["step_ms"])')"
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-140)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fx -o fx -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --backend rccl-native --reserve-cus 32 --grad-exchange activations > $O/prof_fx.log 2>&1 || { echo "prof fx failed"; tail -5 $O/prof_fx.log; exit 1; }
echo "prof_fx: $(grep '^{' $O/prof_fx.log | cut -c1-140)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_g4 -o g4 -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --backend rccl-native --reserve-cus 32 --grad-exchange activations --exchange-groups 4 > $O/prof_g4.log 2>&1 || { echo "prof g4 failed"; tail -5 $O/prof_g4.log; exit 1; }
echo "prof_g4: $(grep '^{' $O/prof_g4.log | cut -c1-140)"
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
cd $R
timeout -k 10 900 python3 -u tools/oom_demo.py > $O/oom.log 2>&1 || { echo "oom demo rc=$?"; tail -5 $O/oom.log; exit 1; }
echo "oom: $(tail -1 $O/oom.log | cut -c1-1500)"
echo done
