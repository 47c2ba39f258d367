#!/bin/bash
# round 6 session 37: kernel traces of the driver's command with the double-buffered head kernels
# (base) and with one load set in both (TDS_HEAD_PF_FWD=0 TDS_HEAD_PF_BWD=0), same box, twice each
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s37
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/base_$i -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/base_$i.log 2>&1 || { echo "base failed"; exit 1; }
  echo "base_$i: $(grep '^{' $O/base_$i.log | cut -c100-160)"
  TDS_HEAD_PF_FWD=0 TDS_HEAD_PF_BWD=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/one_$i -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/one_$i.log 2>&1 || { echo "one failed"; exit 1; }
  echo "one_$i: $(grep '^{' $O/one_$i.log | cut -c100-160)"
done
echo done
