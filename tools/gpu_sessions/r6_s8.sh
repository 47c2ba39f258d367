#!/bin/bash
# round 6 session 8: HEAD validation and evidence -- whole GPU suite + smoke, the driver's command x2,
# the forced activation exchange at W=1 (one group, reserve 0 / 32; four groups, reserve 32, with a
# kernel trace showing the first group's gathers before the last head launch), the transport tune at
# W=1, the OOM demo, a kernel trace of the driver's command and 4 PMC passes of the step
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s8
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t gpu_all 900 tests -m gpu
timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
echo "smoke: $(tail -1 $O/smoke.log)"
for i in 1 2; do
  b drv_$i 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
echo "peak: $(tail -1 $O/drv_1.log | python3 -c 'import json,sys; c=json.loads(sys.stdin.read())["config"]; print(c["peak_mem_gb"])')"
for r in 0 32; do
  b fx_$r 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --backend rccl-native --reserve-cus $r --grad-exchange activations
done
b fx_g4 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --backend rccl-native --reserve-cus 32 --grad-exchange activations --exchange-groups 4
b tune 300 python3 -X faulthandler -u bench.py --gpus 1 --steps 20 --warmup 5 --backend rccl-native --grad-exchange activations --transport-tune
echo "tune: $(tail -1 $O/tune.log | python3 -c 'import json,sys; c=json.loads(sys.stdin.read())["config"]; print(json.dumps(c["preflight"].get("transport"))[:600])')"
timeout -k 10 600 python3 -u tools/oom_demo.py > $O/oom.log 2>&1 || { echo "oom demo rc=$?"; tail -5 $O/oom.log; exit 1; }
echo "oom: $(tail -1 $O/oom.log | cut -c1-600)"
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_fx -o fx -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --backend rccl-native --reserve-cus 32 --grad-exchange activations --exchange-groups 4 > $O/prof_fx.log 2>&1 || { echo "prof fx failed"; tail -5 $O/prof_fx.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
echo "prof: $(grep '^{' $O/prof.log | cut -c1-100)"
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
