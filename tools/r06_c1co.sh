#!/bin/bash
# (the DQN_C1_CO flag and its kernel were removed after the measurement -- rejected)
# Round-6 A/B: conv1 forward with the output channels split over two workgroups on 16x16x32
# MFMAs (this build, DQN_C1_CO=1) vs the one-workgroup-per-sample form (variants/libtsrl_c1old.so
# = -DDQN_C1_CO=0): atari GPU tests on this build, output agreement at 37 and 8192 samples
# (not bit-identical by design: 32-k instead of 16-k MFMA grouping), kernel timings and the
# config-5 bench line, twice interleaved.
timeout -k 10 300 python -u -m pytest tests/test_gpu_atari.py -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider 2>&1 | tail -3 || exit $?
A="python3 tools/atari_kernel_ab.py"
for r in 37 8192; do
  TSRL_LIB_PATH=variants/libtsrl_c1old.so timeout -k 10 120 $A --rows $r --iters 3 --save /tmp/old$r.pt > /dev/null || exit $?
  timeout -k 10 120 $A --rows $r --iters 3 --save /tmp/new$r.pt > /dev/null || exit $?
  echo "rows $r:"; timeout -k 10 60 $A --compare /tmp/old$r.pt /tmp/new$r.pt; echo "compare rc=$?"
done
for r in 1 2; do
  echo "== old"; TSRL_LIB_PATH=variants/libtsrl_c1old.so timeout -k 10 120 $A 2>&1 | head -1 || exit $?
  echo "== co"; timeout -k 10 120 $A 2>&1 | head -1 || exit $?
done
for r in 1 2; do
  echo "== old"; TSRL_LIB_PATH=variants/libtsrl_c1old.so timeout -k 10 300 python3 bench.py --workload atari --steps 3 --warmup 2 --no-cpu-baseline 2>&1 | tail -1 || exit $?
  echo "== co"; timeout -k 10 300 python3 bench.py --workload atari --steps 3 --warmup 2 --no-cpu-baseline 2>&1 | tail -1 || exit $?
done
