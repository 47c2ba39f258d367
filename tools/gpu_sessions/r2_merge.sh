#!/bin/bash
# merged small kernels: tests (kernels, fused, model, big image, full scale), bench, trace
set -u
O=gpurun_out/merge
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_kernels_gpu.py tests/test_fused_gpu.py \
  tests/test_model_gpu.py tests/test_bigimage_gpu.py tests/test_fullscale_gpu.py > $O/tests.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 180 python -u bench.py --steps 40 --warmup 5 > $O/bench.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])'
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
echo prof ok
