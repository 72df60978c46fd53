#!/bin/bash
# Round-6 diagnostics of l1_ring_kernel (mlp_x6.hip L1D builds, wrong results by design):
# where its 180 us per 262144-row minibatch go.  Each variant timed twice, interleaved with the
# shipped build (tools/mlp_kernel_bench.py --only l1_fwd_x6 --ld 384: gathered rows, pitch 384).
B="python3 tools/mlp_kernel_bench.py --only l1_fwd_x6 --ld 384 --iters 30"
VS=${VS:-"1 2 6 7 8"}
for r in 1 2; do
  echo "== base"; timeout -k 10 120 $B || exit $?
  for v in $VS; do
    echo "== L1D=$v"; TSRL_LIB_PATH=variants/libtsrl_l1d$v.so timeout -k 10 120 $B || exit $?
  done
done
