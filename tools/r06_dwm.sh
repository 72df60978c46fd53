#!/bin/bash
# Round-6 decomposition of dw_x6_kernel's time (mlp.hip -DDWM=<bitmask> builds, wrong results by
# design): 1 no split, 2 no MFMA, 4 no loads after the first chunk, 8 no LDS stores after the
# first chunk, 16 no barriers.  Each twice, interleaved with the shipped build.
B="python3 tools/mlp_kernel_bench.py --only dw --ld 384 --iters 30"
VS=${VS:-"1 2 4 8 16 6 14 30"}
for r in 1 2; do
  echo "== base"; timeout -k 10 120 $B || exit $?
  for v in $VS; do
    echo "== DWM=$v"; TSRL_LIB_PATH=variants/libtsrl_d$v.so timeout -k 10 120 $B || exit $?
  done
done
