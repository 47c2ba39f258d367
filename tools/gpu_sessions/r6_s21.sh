#!/bin/bash
# round 6 session 21 (diagnostic): the >2 GiB one-step test on the fp16-g2m build and on the previous
# HEAD (_C_prev.so): conv2 bias-gradient error against its bound, printed
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s21
mkdir -p $O
cd $GRAFT_REPO_ROOT
for v in new prev; do
  if [ $v = new ]; then V=; else V=$v; fi
  TDS_SO_VARIANT=$V timeout -k 10 300 python -u -m pytest tests/test_bigimage_gpu.py -m gpu -x -q -s --timeout 240 --timeout-method thread -k beyond > $O/big_$v.log 2>&1
  echo "$v rc=$?: $(grep -E 'conv2 bias|fc tail|passed|failed' $O/big_$v.log | tr '\n' ' ' | cut -c1-400)"
done
echo done
