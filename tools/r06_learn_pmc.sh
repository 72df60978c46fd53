#!/bin/bash
# Round-6 HBM counter passes over one 262144-row PPO minibatch on the final tree
# (tools/mlp_kernel_bench.py --only minibatch --ld 384), FETCH_SIZE and WRITE_SIZE in separate
# runs, each summarised on the box (tools/pmc_summary.py) and deleted.
export TMPDIR=/tmp
P="timeout -s KILL 120 rocprofv3"
S="python3 tools/pmc_summary.py"
tools/gpu_run.sh \
  "pmc_f:150:$P --pmc FETCH_SIZE -d gpurun_out/pmc_f -o run -- python3 tools/mlp_kernel_bench.py --only minibatch --ld 384 && $S gpurun_out/pmc_f/run_results.db > gpurun_out/pmc_f.txt && rm -rf gpurun_out/pmc_f" \
  "pmc_w:150:$P --pmc WRITE_SIZE -d gpurun_out/pmc_w -o run -- python3 tools/mlp_kernel_bench.py --only minibatch --ld 384 && $S gpurun_out/pmc_w/run_results.db > gpurun_out/pmc_w.txt && rm -rf gpurun_out/pmc_w" \
  "$@"
