#!/bin/bash
# round 6 session 12: conv2 forward epilogue A/B -- the argmax-code words by one byte permute of
# the ballot's 32-bit half (instead of a per-lane 64-bit shift) and the y2h values written as
# per-lane half-words (instead of DPP-paired words): default build = both, _C_f2a2.so = the
# permute only, _C_f2old.so = neither.  GPU tests of the default build first; isolated op times,
# the driver's command and one VALU/MFMA counter pass per build.
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s12
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t c2 400 tests/test_fused_gpu.py tests/test_model_gpu.py tests/test_fullscale_plan_gpu.py tests/test_determinism_gpu.py -m gpu
for v in new f2a2 f2old new f2a2 f2old; do
  if [ $v = new ]; then V=; else V=$v; fi
  OP_ONLY=conv2_fwd op c2_$v TDS_SO_VARIANT=$V
done
for v in new f2a2 f2old new f2a2 f2old; do
  if [ $v = new ]; then V=; else V=$v; fi
  b drv_$v 200 env TDS_SO_VARIANT=$V python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
cd /tmp && export TMPDIR=/tmp && cd $R
for v in new f2old; do
  if [ $v = new ]; then V=; else V=$v; fi
  TDS_SO_VARIANT=$V timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_$v -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  echo "pmc $v ok"
done
echo done
