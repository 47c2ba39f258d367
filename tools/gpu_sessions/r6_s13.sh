#!/bin/bash
# round 6 session 13: conv2 forward -- a max-only window path for waves whose 16 channels all have
# gamma2 > 0 (wave-uniform) and the argmax code bits from per-comparison ballots by scalar logic
# (default build) against the same without the max-only path (_C_f2noplain.so); GPU tests first
set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r6s13
mkdir -p $O
source $GRAFT_REPO_ROOT/tools/gpu_sessions/lib.sh
t c2 400 tests/test_fused_gpu.py tests/test_model_gpu.py tests/test_fullscale_plan_gpu.py tests/test_determinism_gpu.py -m gpu
for v in new noplain new noplain; do
  if [ $v = new ]; then V=; else V=f2$v; fi
  OP_ONLY=conv2_fwd op c2_$v TDS_SO_VARIANT=$V
done
for v in new noplain new noplain; do
  if [ $v = new ]; then V=; else V=f2$v; fi
  b drv_$v 200 env TDS_SO_VARIANT=$V python3 -u bench.py --gpus 1 --steps 20 --warmup 5
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_new -o run -- python3 $R/bench.py --steps 2 --warmup 1 > $O/pmc_new.log 2>&1 || { echo "pmc failed"; exit 1; }
echo done
