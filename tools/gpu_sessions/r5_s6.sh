#!/bin/bash
# round 5 session 6: (1) GPU tests incl. the exchange's ya encoder (bitwise vs the written X), the
# forced overflow step, and the head forward applying the deferred exchange update; (2) conv2
# backward staging breakdown (diag build: 16 full, 17 no staging, 28 staging alone, 60 staging alone
# w/o global loads, 92 staging alone w/o BN2/pool math, 48 full w/o staging loads, 80 full w/o
# staging math); (3) driver command; forced activation exchange at W=1 with / without the CU
# split, and with the separate update sweep + dense X (TDS_FUSED_FIN=0); (4) one-GPU rehearsal of a
# 200 MB copy beside the backward on the copy engines vs the blit kernel; (5) trace of the forced
# exchange step (last: its teardown aborts under rocprofv3)
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s6
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_model_gpu.py tests/test_comm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -40 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
op() {
  local name=$1; shift
  timeout -k 10 240 env "$@" python3 -u tools/micro/step_ops_timing.py --iters 10 --only conv2_bwd > $O/op_$name.log 2>&1 || { echo "op $name rc=$?"; tail -5 $O/op_$name.log; exit 1; }
  echo "op $name: $(grep -v amdgpu.ids $O/op_$name.log | grep -v '^{' | tr '\n' ' ' | cut -c1-300)"
}
op base TDS_SO_VARIANT=
for d in 16 17 28 60 92 48 80; do op d$d TDS_SO_VARIANT=diag TDS_CONV2_DIAG=$d; done
b() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -5 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); c=r["config"]; print(r["ms_per_step"], r["value"], c.get("x_exchange"), c.get("sim_sdma"))')"
}
b drv1 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
b xa32 240 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
b xa0 240 python3 -u bench.py --backend rccl-native --reserve-cus 0 --grad-exchange activations --steps 20 --warmup 5
b xa32sep 240 env TDS_FUSED_FIN=0 python3 -u bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5
b sdma_nocu 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --sim-sdma-mb 200 --sim-sdma-engine nocu
b sdma_blit 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --sim-sdma-mb 200 --sim-sdma-engine blit
b drv2 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_sdma -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --sim-sdma-mb 200 --sim-sdma-engine nocu > $O/trace_sdma.log 2>&1 || { echo "trace sdma rc=$?"; tail -5 $O/trace_sdma.log; exit 1; }
echo "trace_sdma ok"
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_xa -o run -- \
  python3 $R/bench.py --backend rccl-native --reserve-cus 32 --grad-exchange activations --steps 20 --warmup 5 > $O/trace_xa.log 2>&1
echo "trace_xa rc=$? (the exit abort under rocprofv3 is known; the csv is written before it)"
