#!/bin/bash
# Round-6 counter passes over the LDS-staged config-5 trunk kernels (tools/atari_kernel_ab.py,
# 8192 samples, 5 launches each): SQ issue / wait / MFMA-busy, LDS, and HBM FETCH / WRITE, one
# counter group per run; each database summarised on the box and deleted.
export TMPDIR=/tmp
P="timeout -s KILL 120 rocprofv3"
S="python3 tools/pmc_summary.py"
A="python3 tools/atari_kernel_ab.py --iters 2"
tools/gpu_run.sh \
  "pa_sq:150:$P --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d /tmp/pa_sq -o run -- $A && $S /tmp/pa_sq/run_results.db dqn > gpurun_out/pa_sq.txt && rm -rf /tmp/pa_sq" \
  "pa_lds:150:$P --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVES -d /tmp/pa_lds -o run -- $A && $S /tmp/pa_lds/run_results.db dqn > gpurun_out/pa_lds.txt && rm -rf /tmp/pa_lds" \
  "pa_f:150:$P --pmc FETCH_SIZE -d /tmp/pa_f -o run -- $A && $S /tmp/pa_f/run_results.db dqn > gpurun_out/pa_f.txt && rm -rf /tmp/pa_f" \
  "pa_w:150:$P --pmc WRITE_SIZE -d /tmp/pa_w -o run -- $A && $S /tmp/pa_w/run_results.db dqn > gpurun_out/pa_w.txt && rm -rf /tmp/pa_w"
