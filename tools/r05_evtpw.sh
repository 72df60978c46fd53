#!/bin/bash
# Round-5 A/B: the layer-1 kernel over contiguous rows (process_fn's 2M-row evaluation chunks)
# with one workgroup per CU walking all its tiles (default) vs at most 4 tiles per workgroup
# (TSRL_L1_TPW=4, the previous grid): parity, the eval chunk time, then the bench update time.
export TMPDIR=/tmp
T="python -u -m pytest -q -x -rf --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu"
K="python tools/mlp_kernel_bench.py --iters 10 --only eval"
B="python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline"
tools/gpu_run.sh \
  "t_tpw:600:$T tests/test_gpu_mlp.py tests/test_gpu_ppo.py tests/test_gpu_rollout.py tests/test_gpu_wide.py tests/test_gpu_fullsize.py" \
  "ab_k:300:for v in new old new old; do echo == \$v; if [ \$v = old ]; then export TSRL_L1_TPW=4; else unset TSRL_L1_TPW; fi; timeout -k 10 100 $K || exit 3; done" \
  "ab_b:700:for v in new old new old; do echo == \$v; if [ \$v = old ]; then export TSRL_L1_TPW=4; else unset TSRL_L1_TPW; fi; timeout -k 10 150 $B 2>&1 | grep -E '^# iter 2' || exit 3; done" \
  "$@"
