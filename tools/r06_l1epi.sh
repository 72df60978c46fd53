#!/bin/bash
# Round-6: l1_ring_kernel epilogue cost -- shipped build (tanh / identity), -DL1M=64 (the same
# stores issued lane-contiguous: 1 KB per instruction, wrong layout for the consumers),
# -DL1M=16 (no epilogue).  Two passes, interleaved.
B="python3 tools/mlp_kernel_bench.py --only l1_fwd_x6 --ld 384 --iters 30"
for r in 1 2; do
  echo "== base"; timeout -k 10 120 $B || exit $?
  echo "== base identity"; timeout -k 10 120 $B --act 0 || exit $?
  echo "== L1M=64"; TSRL_LIB_PATH=variants/libtsrl_m64.so timeout -k 10 120 $B || exit $?
  echo "== L1M=64 identity"; TSRL_LIB_PATH=variants/libtsrl_m64.so timeout -k 10 120 $B --act 0 || exit $?
  echo "== L1M=16"; TSRL_LIB_PATH=variants/libtsrl_m16.so timeout -k 10 120 $B || exit $?
done
