#!/bin/bash
# Round-6 A/B: conv1 weight gradient with packed 4-byte split-plane stores of the gradient rows
# (this build) vs the 2-byte stores (variants/libtsrl_w0.so = HEAD's dqn_conv.hip); atari GPU
# tests on this build, outputs compared at 37 / 8192 samples, timings twice interleaved.
timeout -k 10 300 python -u -m pytest tests/test_gpu_atari.py -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2 || exit $?
A="python3 tools/atari_kernel_ab.py"
for r in 37 8192; do
  TSRL_LIB_PATH=variants/libtsrl_w0.so timeout -k 10 120 $A --rows $r --iters 3 --save /tmp/old$r.pt > /dev/null || exit $?
  timeout -k 10 120 $A --rows $r --iters 3 --save /tmp/new$r.pt > /dev/null || exit $?
  echo "rows $r:"; timeout -k 10 60 $A --compare /tmp/old$r.pt /tmp/new$r.pt; echo "compare rc=$?"
done
for r in 1 2; do
  echo "== w0"; TSRL_LIB_PATH=variants/libtsrl_w0.so timeout -k 10 120 $A | grep wgrad || exit $?
  echo "== packed"; timeout -k 10 120 $A | grep wgrad || exit $?
done
