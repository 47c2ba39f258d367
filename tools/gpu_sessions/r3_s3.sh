#!/bin/bash
# round 3: where the exchange's side work should run (W=1, exchange forced, 32 CUs split off):
# on the reserved CUs (TDS_SIDE_CUS=comm) vs unmasked (any) vs compute CUs; then whether a kernel
# trace survives CU-masked streams -- last, since a crash ends the session
set -u
O=gpurun_out/r3s3
mkdir -p $O
b() {
  local name=$1; shift
  timeout -k 10 200 python -u bench.py "$@" > $O/$name.log 2>&1 || { echo "$name rc=$?"; tail -20 $O/$name.log; exit 1; }
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"], r["config"]["fc_grad"], r["config"]["reserve_cus"])')"
}
# the tests whose bounds moved to the TF32-reference class (fp16x2 conv2)
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_multirank_gpu.py tests/test_bigimage_gpu.py -v -s \
  --timeout 400 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "FAILED|passed|failed" $O/tests.log | tail -12
[ $rc -le 1 ] || { echo "tests rc=$rc"; tail -40 $O/tests.log; exit 1; }
timeout -k 10 200 python -u tools/micro/step_ops_timing.py > $O/ops.log 2>&1 || { echo "ops rc=$?"; tail -20 $O/ops.log; exit 1; }
tail -1 $O/ops.log
b local_r32 --steps 30 --warmup 5 --reserve-cus 32
for side in comm any compute; do
  TDS_SIDE_CUS=$side b act_$side --steps 30 --warmup 5 --grad-exchange activations --reserve-cus 32
  TDS_SIDE_CUS=$side b shd_$side --steps 30 --warmup 5 --grad-exchange sharded --reserve-cus 32
done
(cd /tmp && TMPDIR=/tmp timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/actzs_prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --grad-exchange activations > $GRAFT_REPO_ROOT/$O/actzs_prof.log 2>&1) \
  || { echo "act_zs prof rc=$?"; tail -20 $O/actzs_prof.log; exit 1; }
echo "act_zs prof ok"
timeout -k 10 120 python -u tools/micro/masked_stream_probe.py > $O/probe_bare.log 2>&1 || { echo "probe bare rc=$?"; tail -20 $O/probe_bare.log; exit 1; }
tail -1 $O/probe_bare.log
cd /tmp && export TMPDIR=/tmp
PYTHONFAULTHANDLER=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/probe_prof -o run -- \
  python3 $GRAFT_REPO_ROOT/tools/micro/masked_stream_probe.py > $GRAFT_REPO_ROOT/$O/probe_prof.log 2>&1 || { echo "probe under rocprof rc=$?"; tail -30 $GRAFT_REPO_ROOT/$O/probe_prof.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/$O/probe_prof.log
