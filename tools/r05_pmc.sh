#!/bin/bash
# Round-5 HBM counter passes (one counter block per run, each under its own time limit):
# the fused collect step (tools/collect_step_bench.py) and one 262144-row PPO minibatch
# (tools/mlp_kernel_bench.py --only minibatch --ld 384); summaries: tools/pmc_summary.py,
# tools/pmc_learn.py.
export TMPDIR=/tmp
tools/gpu_run.sh \
  "pmc_cf:150:timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_cf -o run -- python3 tools/collect_step_bench.py --steps 64 --reps 1" \
  "pmc_cw:150:timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_cw -o run -- python3 tools/collect_step_bench.py --steps 64 --reps 1" \
  "pmc_f:150:timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o run -- python3 tools/mlp_kernel_bench.py --only minibatch --ld 384" \
  "pmc_w:150:timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o run -- python3 tools/mlp_kernel_bench.py --only minibatch --ld 384" \
  "$@"
