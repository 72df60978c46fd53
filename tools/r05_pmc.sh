#!/bin/bash
# Round-5 HBM counter passes (one counter block per run, each under its own time limit):
# the fused collect step (tools/collect_step_bench.py) and one 262144-row PPO minibatch
# (tools/mlp_kernel_bench.py --only minibatch --ld 384).  Each database is summarised on the
# box (tools/pmc_summary.py) and deleted, so gpurun_out/ stays small.
export TMPDIR=/tmp
P="timeout -s KILL 120 rocprofv3"
S="python3 tools/pmc_summary.py"
tools/gpu_run.sh \
  "pmc_cf:150:$P --pmc FETCH_SIZE -d gpurun_out/pmc_cf -o run -- python3 tools/collect_step_bench.py --steps 64 --reps 1 && $S gpurun_out/pmc_cf/run_results.db collect_box > gpurun_out/pmc_cf.txt && rm -rf gpurun_out/pmc_cf" \
  "pmc_cw:150:$P --pmc WRITE_SIZE -d gpurun_out/pmc_cw -o run -- python3 tools/collect_step_bench.py --steps 64 --reps 1 && $S gpurun_out/pmc_cw/run_results.db collect_box > gpurun_out/pmc_cw.txt && rm -rf gpurun_out/pmc_cw" \
  "pmc_f:150:$P --pmc FETCH_SIZE -d gpurun_out/pmc_f -o run -- python3 tools/mlp_kernel_bench.py --only minibatch --ld 384 && $S gpurun_out/pmc_f/run_results.db > gpurun_out/pmc_f.txt && rm -rf gpurun_out/pmc_f" \
  "pmc_w:150:$P --pmc WRITE_SIZE -d gpurun_out/pmc_w -o run -- python3 tools/mlp_kernel_bench.py --only minibatch --ld 384 && $S gpurun_out/pmc_w/run_results.db > gpurun_out/pmc_w.txt && rm -rf gpurun_out/pmc_w" \
  "$@"
