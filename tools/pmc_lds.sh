#!/bin/bash
# SQ stall / LDS counters on one PPO minibatch's kernels (tools/mlp_kernel_bench.py --only
# minibatch), one rocprofv3 --pmc pass per counter group (MI355X_MICROARCH.md: <= 8 SQ each).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1 || true
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $R/gpurun_out/pmc$i -o run --output-format csv -- \
      python3 $R/tools/mlp_kernel_bench.py --only minibatch --iters 3 > $R/gpurun_out/pmc$i.log 2>&1 || exit $?
done
