#!/bin/bash
# Round-5: captured learn epochs write each minibatch's loss terms straight into the graph's
# [n_minibatch, 4] output (no copy node per minibatch): parity of the graph / data-parallel
# learn paths, then config 2 (2048-row minibatches, graph-replayed epochs) twice.
export TMPDIR=/tmp
T="python -u -m pytest -q -x -rf --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu"
B="python3 bench.py --workload small --steps 3 --warmup 2 --no-cpu-baseline"
tools/gpu_run.sh \
  "t_terms:600:$T tests/test_gpu_ppo.py tests/test_gpu_trainer.py tests/test_gpu_sched.py tests/test_gpu_a_dist.py tests/test_gpu_a0_nccl.py tests/test_gpu_capture_gc.py" \
  "ab:400:for v in 1 2; do timeout -k 10 150 $B > gpurun_out/b\$v.log 2>&1 || exit 3; grep -E '^# iter 2|^\{' gpurun_out/b\$v.log | cut -c1-200; done" \
  "$@"
