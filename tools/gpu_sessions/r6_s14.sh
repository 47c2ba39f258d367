#!/bin/bash
# round 6 session 14: conv2 backward staging -- the argmax routing of the pooled gradient by
# bit-field selects (v_bitop3 on the code bits sign-extended to masks) instead of code compares and
# selects (default build) against _C_brold.so (-D TDS_BR_OLD_SEL); GPU tests first
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s14
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t c2b 400 tests/test_fused_gpu.py tests/test_model_gpu.py tests/test_fullscale_plan_gpu.py tests/test_determinism_gpu.py tests/test_bigimage_gpu.py -m gpu
for v in new old new old; do
  if [ $v = new ]; then V=; else V=brold; fi
  OP_ONLY=conv2_bwd op c2b_$v TDS_SO_VARIANT=$V
done
for v in new old new old; do
  if [ $v = new ]; then V=; else V=brold; fi
  b drv_$v 200 env TDS_SO_VARIANT=$V python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
cd /tmp && export TMPDIR=/tmp && cd $R
for v in new old; do
  if [ $v = new ]; then V=; else V=brold; fi
  TDS_SO_VARIANT=$V timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_$v -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
done
echo done
