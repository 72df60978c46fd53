#!/bin/bash
# dW1 kernel A/B at the benchmark shape: the in-tree library, then each named variant
# (variants/libtsrl_<name>.so from tools/build_variant.sh mlp.hip -D...).
set -o pipefail
for v in main "$@" main "$@"; do
  unset TSRL_LIB_PATH
  [ $v = main ] || export TSRL_LIB_PATH=variants/libtsrl_$v.so
  echo "== $v"
  timeout -k 10 120 python tools/mlp_kernel_bench.py --iters 20 --only dw || exit $?
  timeout -k 10 120 python tools/mlp_kernel_bench.py --iters 10 --only minibatch || exit $?
done
