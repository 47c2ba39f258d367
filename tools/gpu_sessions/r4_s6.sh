#!/bin/bash
# round 4 session 6: evidence -- kernel trace of the driver's bench command, 4 PMC passes of the
# default step (incl. the layer-1 backward's LDS bank conflicts), zs ratio on the bench noise and
# on SyntheticMNIST digits at 3000^2, mnist_onegpu.py vs bench.py on one box, the W=1 forced-exchange
# traces (no host wait between the head backward and the conv2 backward), the OOM demo at 18000^2
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s6
mkdir -p $O
cd $R
timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 20 --step-times > $O/w20.log 2>&1 || { echo "w20 rc=$?"; exit 1; }
python3 -c "import json,sys; r=json.loads(open('$O/w20.log').read().strip().splitlines()[-1]); s=r['config']['step_ms']; print('warmup20', r['ms_per_step'], s[:4], s[-3:])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo "trace ok: $(tail -1 $O/trace.log | cut -c80-200)"
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
cd $R
for d in noise mnist; do
  timeout -k 10 300 python3 -u tools/x_sparsity.py --data $d --train-steps 20 > $O/xs_$d.log 2>&1 || { echo "xs $d rc=$?"; tail -5 $O/xs_$d.log; exit 1; }
  echo "xs $d: $(tail -1 $O/xs_$d.log | cut -c1-400)"
done
timeout -k 10 300 python3 -u bench.py > $O/bench_default.log 2>&1 || { echo "bench rc=$?"; exit 1; }
echo "bench 100: $(tail -1 $O/bench_default.log | cut -c80-200)"
timeout -k 10 300 python3 -u mnist_onegpu.py --epochs 1 --max-steps 100 --json > $O/onegpu.log 2>&1 || { echo "onegpu rc=$?"; tail -5 $O/onegpu.log; exit 1; }
echo "onegpu: $(tail -1 $O/onegpu.log)"
cd /tmp
for gx in activations sharded; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/ex_$gx -o run -- \
    python3 $R/bench.py --steps 8 --warmup 3 --backend rccl-native --grad-exchange $gx > $O/ex_$gx.log 2>&1 || { echo "ex $gx rc=$?"; tail -5 $O/ex_$gx.log; exit 1; }
  echo "ex $gx: $(tail -1 $O/ex_$gx.log | cut -c80-200)"
done
cd $R
timeout -k 10 600 python3 -u tools/oom_demo.py --image-size 18000 > $O/oom.log 2>&1 || { echo "oom rc=$?"; tail -5 $O/oom.log; exit 1; }
echo "oom: $(tail -1 $O/oom.log)"
