#!/bin/bash
# Shared helpers of the round-5 GPU session scripts (source after setting O, the output dir).
# Every GPU step runs under its own time limit; a crash-class exit (abort, segfault, time limit)
# ends the session, an ordinary test failure is reported and the session goes on measuring.
R=$GRAFT_REPO_ROOT
cd $R

crash_rc() {  # 124 timeout, 134 abort, 137 kill, 139 segfault
  case $1 in 124|134|137|139) return 0 ;; *) return 1 ;; esac
}

# t NAME SECONDS pytest-args...: a pytest run; failures are printed, crashes end the session
t() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc: $(tail -1 $O/$name.log)"
  if [ $rc -ne 0 ]; then grep -E "^(E |FAILED|>)" $O/$name.log | head -20; fi
  if crash_rc $rc; then echo "crash-class exit: stopping"; exit 1; fi
  return 0
}

# op NAME env...: the isolated conv2 backward on a real step's tensors (median of 5 x 10 calls)
op() {
  local name=$1; shift
  timeout -k 10 240 env "$@" python3 -u tools/micro/step_ops_timing.py --iters 10 --only ${OP_ONLY:-conv2_bwd} > $O/op_$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "op $name rc=$rc"; tail -5 $O/op_$name.log; exit 1; fi
  echo "op $name: $(grep -v amdgpu.ids $O/op_$name.log | grep -v '^{' | tr '\n' ' ' | cut -c1-400)"
}

# b NAME SECONDS cmd...: a bench run; prints ms/step, images/s and the exchange / sdma config
b() {
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $O/$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -5 $O/$name.log; exit 1; fi
  echo "$name: $(tail -1 $O/$name.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); c=r["config"]; print(r["ms_per_step"], r["value"], c.get("fc_grad"), c.get("x_exchange"), c.get("sim_sdma"))')"
}
