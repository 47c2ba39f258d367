#!/bin/bash
# kernel traces of the exchanged fc-gradient paths at world 1 (no CU split: rocprofv3 + masked streams segfaulted)
set -u
O=gpurun_out/paths_prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for p in sharded activations; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/$p -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 3 --backend rccl-native --grad-exchange $p --reserve-cus 0 > $GRAFT_REPO_ROOT/$O/$p.log 2>&1 || { echo "prof $p rc=$?"; exit 1; }
  tail -1 $GRAFT_REPO_ROOT/$O/$p.log | cut -c1-300
done
echo prof ok
