#!/bin/bash
# Tail-kernel A/B timings of variants at the benchmark shape.
set -o pipefail
for v in main t4 main t4; do
  if [ $v = main ]; then unset TSRL_LIB_PATH; else export TSRL_LIB_PATH=variants/libtsrl_$v.so; fi
  echo "== $v"
  timeout -k 10 120 python tools/mlp_kernel_bench.py --iters 20 --only tail || exit $?
done
