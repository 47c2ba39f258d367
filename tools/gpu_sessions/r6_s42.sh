#!/bin/bash
# round 6 session 42: kernel traces of the driver's command with the head backward's band 2 and 4
# (TDS_HEAD_BAND_B, temporary), same box, twice each
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s42
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for i in 1 2; do
  for bnd in 2 4; do
    TDS_HEAD_BAND_B=$bnd timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b${bnd}_$i -o run -- python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/b${bnd}_$i.log 2>&1 || { echo "trace failed"; exit 1; }
    echo "b${bnd}_$i ok"
  done
done
echo done
