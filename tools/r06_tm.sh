#!/bin/bash
# Round-6 decomposition of the ppo_tail16 kernels (mlp.hip -DTM=<bitmask> builds, wrong results
# by design): 1 no dZ1 stores, 2 no per-row input loads, 4 no layer-2/3 weight-gradient
# accumulation.  Both nets + the reduction (tools/mlp_kernel_bench.py --only tail), twice.
B="python3 tools/mlp_kernel_bench.py --only tail --ld 384 --iters 30"
for r in 1 2; do
  echo "== base"; timeout -k 10 120 $B || exit $?
  for v in 1 2 4 7; do
    echo "== TM=$v"; TSRL_LIB_PATH=variants/libtsrl_t$v.so timeout -k 10 120 $B || exit $?
  done
done
