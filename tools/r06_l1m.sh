#!/bin/bash
# Round-6 decomposition of l1_ring_kernel's time (mlp_x6.hip -DL1M=<bitmask> builds, wrong
# results by design): 1 no split, 2 no MFMA, 4 no X reload, 8 no W reload, 16 no epilogue,
# 32 W fragments reused across the chunk.  Each variant twice, interleaved with the shipped build.
B="python3 tools/mlp_kernel_bench.py --only l1_fwd_x6 --ld 384 --iters 30"
VS=${VS:-"2 6 14 30 31 16 32 12 48"}
for r in 1 2; do
  echo "== base"; timeout -k 10 120 $B || exit $?
  for v in $VS; do
    echo "== L1M=$v"; TSRL_LIB_PATH=variants/libtsrl_m$v.so timeout -k 10 120 $B || exit $?
  done
done
