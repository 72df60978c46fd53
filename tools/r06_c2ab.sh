#!/bin/bash
# (the build flags this recipe names were removed after the measurement; the recipe documents
# how the committed log was produced -- rebuild the variants from the commit it cites to rerun)
# Round-6 A/B: conv2 data gradient with two classes per 8-wave workgroup (this build) vs one
# class per 4-wave workgroup (variants/libtsrl_n1.so = -DDQN_C2_NCL=1) and the gathered form
# (variants/libtsrl_g.so); atari GPU tests on this build, bit-identity at 37 / 8192 samples.
timeout -k 10 300 python -u -m pytest tests/test_gpu_atari.py -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2 || exit $?
A="python3 tools/atari_kernel_ab.py"
for r in 37 8192; do
  TSRL_LIB_PATH=variants/libtsrl_g.so timeout -k 10 120 $A --rows $r --iters 3 --save /tmp/old$r.pt > /dev/null || exit $?
  timeout -k 10 120 $A --rows $r --iters 3 --save /tmp/new$r.pt > /dev/null || exit $?
  echo "rows $r:"; timeout -k 10 60 $A --compare /tmp/old$r.pt /tmp/new$r.pt; echo "compare rc=$?"
done
for r in 1 2; do
  echo "== gather"; TSRL_LIB_PATH=variants/libtsrl_g.so timeout -k 10 120 $A | grep dgrad || exit $?
  echo "== ncl1"; TSRL_LIB_PATH=variants/libtsrl_n1.so timeout -k 10 120 $A | grep dgrad || exit $?
  echo "== ncl2"; timeout -k 10 120 $A | grep dgrad || exit $?
done
