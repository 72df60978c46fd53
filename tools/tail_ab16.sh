#!/bin/bash
# Tail A/B (round 5): the in-tree library (16-row tail at two waves per SIMD) against a
# -DTAIL16=0 build (variants/libtsrl_tail32.so, tools/build_variant.sh), after the learn
# tests on the in-tree library.
export TMPDIR=/tmp
T="python -u -m pytest -q -x -rf --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu"
tools/gpu_run.sh \
  "t_learn:600:$T tests/test_gpu_mlp.py tests/test_gpu_ppo.py tests/test_gpu_sched.py tests/test_gpu_optim.py" \
  "ab_tail:600:for v in main tail32 main tail32; do unset TSRL_LIB_PATH; [ \$v = main ] || export TSRL_LIB_PATH=variants/libtsrl_\$v.so; echo == \$v; timeout -k 10 100 python tools/mlp_kernel_bench.py --iters 20 --only tail --ld 384 || exit \$?; timeout -k 10 100 python tools/mlp_kernel_bench.py --iters 10 --only minibatch --ld 384 || exit \$?; done" \
  "$@"
