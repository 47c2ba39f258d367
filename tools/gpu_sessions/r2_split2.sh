#!/bin/bash
# CU split moved into init_process_group: comm + bench tests, bench variants
set -u
O=gpurun_out/split2
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_comm_gpu.py tests/test_bench_gpu.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
b() {
  local name=$1; shift
  timeout -k 10 150 python -u bench.py --steps 60 --warmup 8 "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); c=r["config"]; print(r["value"], r["ms_per_step"], c["reserve_cus"], c["rccl_max_ctas"], c.get("sim_comm"))')"
}
b base
b r32_sim3000 --reserve-cus 32 --sim-comm-us 3000 --sim-comm-ctas 32
b native_ex_r32 --grad-exchange activations --reserve-cus 32
for k in 1 2 3; do
  b def_$k
  TDS_SO_VARIANT=nt b nt_$k
done
timeout -k 10 150 python -u tools/micro/step_ops_timing.py --iters 10 > $O/ops_def.log 2>&1 && tail -1 $O/ops_def.log
TDS_SO_VARIANT=nt timeout -k 10 150 python -u tools/micro/step_ops_timing.py --iters 10 > $O/ops_nt.log 2>&1 && tail -1 $O/ops_nt.log
