#!/bin/bash
# Round-5: adaptive tiles per workgroup in the layer-1 ring kernel (small minibatches: config 2)
# -- parity (mlp / padded / sched tests), config 2 bench twice, the headline bench once -- and
# the dW1 split-count A/B (ns256 / ns208 vs 168).
export TMPDIR=/tmp
T="python -u -m pytest -q -x -rf --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu"
B="python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline"
tools/gpu_run.sh \
  "t_s:400:$T tests/test_gpu_mlp.py tests/test_gpu_padded.py tests/test_gpu_sched.py tests/test_gpu_trainer.py" \
  "b_small:300:$B --workload small" \
  "b_small2:300:$B --workload small" \
  "b_head:300:$B" \
  "ab_dw:600:tools/dw_ab.sh ns256 ns208" \
  "$@"
