#!/bin/bash
# round 4 session 27: layer-1 conv LDS row stride 81 (odd; 80 put the two lane groups of a
# 32-lane half on the same 16 banks) and the conv2 forward's conflict-free y2h store read
# (F2_QPX) -- fused/model tests, then the driver's command alternating with the stride-80 and
# QPX-off variant builds on the same box, a kernel trace and the LDS PMC pass
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4s27
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $O/tests.log | head -20; exit 1; }
b() {
  local name=$1; shift
  timeout -k 10 200 env "$@" python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["ms_per_step"], r["value"])')"
}
b new_1 TDS_SO_VARIANT=
b x80_1 TDS_SO_VARIANT=l1x80
b q0_1 TDS_SO_VARIANT=f2q0
b new_2 TDS_SO_VARIANT=
b x80_2 TDS_SO_VARIANT=l1x80
b q0_2 TDS_SO_VARIANT=f2q0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace.log; exit 1; }
echo trace ok
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE \
  --output-format csv -d $O/pd -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $O/pd.log 2>&1 && echo pd ok
