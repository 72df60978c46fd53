#!/bin/bash
# (the build flags this recipe names were removed after the measurement; the recipe documents
# how the committed log was produced -- rebuild the variants from the commit it cites to rerun)
# Round-6 A/B: conv1 forward and conv2 data gradient from LDS-staged samples (this build) vs the gathered form
# (variants/libtsrl_g.so = -DDQN_C1_GATHER=1 -DDQN_C2_GATHER=1): atari GPU tests on this build, bit-identity of
# the outputs at 8192 and 37 samples, timings twice interleaved.
timeout -k 10 300 python -u -m pytest tests/test_gpu_atari.py -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider 2>&1 | tail -3 || exit $?
A="python3 tools/atari_kernel_ab.py"
for r in 37 8192; do
  TSRL_LIB_PATH=variants/libtsrl_g.so timeout -k 10 120 $A --rows $r --iters 3 --save /tmp/old$r.pt > /dev/null || exit $?
  timeout -k 10 120 $A --rows $r --iters 3 --save /tmp/new$r.pt > /dev/null || exit $?
  echo "rows $r:"; timeout -k 10 60 $A --compare /tmp/old$r.pt /tmp/new$r.pt; echo "compare rc=$?"
done
for r in 1 2; do
  echo "== gather"; TSRL_LIB_PATH=variants/libtsrl_g.so timeout -k 10 120 $A || exit $?
  echo "== lds"; timeout -k 10 120 $A || exit $?
done
