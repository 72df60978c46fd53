#!/bin/bash
# (the build flags this recipe names were removed after the measurement; the recipe documents
# how the committed log was produced -- rebuild the variants from the commit it cites to rerun)
# Round-6 decomposition of the LDS-staged config-5 trunk kernels (dqn_conv.hip -DDQM=<bit>
# builds, wrong results by design): conv1 forward -- 1 no MFMA, 2 no byte->bf16 conversion,
# 4 no output stores, 8 no frame staging; conv2 data gradient -- 1 no MFMA, 2 no z1 mask loads,
# 4 no dx stores, 8 no split/LDS staging of gy2, 16 no gy2 loads.  Two passes, one box.
A="python3 tools/atari_kernel_ab.py --iters 20"
for r in 1 2; do
  echo "== base"; timeout -k 10 120 $A | grep -v wgrad || exit $?
  for m in 1 2 4 8 16; do
    echo "== DQM=$m"; TSRL_LIB_PATH=variants/libtsrl_q$m.so timeout -k 10 120 $A | grep -v wgrad || exit $?
  done
done
