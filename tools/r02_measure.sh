#!/bin/bash
# Round-2 measurement pass (one GPU call): GPU tests, headline bench, rocprof kernel stats of
# the bench, and PMC HBM-byte passes (FETCH_SIZE, WRITE_SIZE in separate runs) over one
# learn minibatch's kernels (tools/mlp_kernel_bench.py --only minibatch).
export TMPDIR=/tmp
tools/gpu_run.sh \
  "tests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "bench:240:python -u bench.py" \
  "prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 2" \
  "pmc_f:120:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o run -- python3 tools/mlp_kernel_bench.py --only minibatch --iters 3" \
  "pmc_w:120:timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o run -- python3 tools/mlp_kernel_bench.py --only minibatch --iters 3"
