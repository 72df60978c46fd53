#!/bin/bash
# (the build flags this recipe names were removed after the measurement; the recipe documents
# how the committed log was produced -- rebuild the variants from the commit it cites to rerun)
# Round-6 A/B: dw_x6 staging with pair loads + DPP swap (this build) vs the round-5 staging
# (variants/libtsrl_pl0.so = -DDWX6_PAIRLD=0); MLP / PPO tests on this build first.
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_ppo.py tests/test_gpu_wide.py tests/test_gpu_padded.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider 2>&1 | tail -3 || exit $?
B="python3 tools/mlp_kernel_bench.py --ld 384 --iters 30"
for r in 1 2; do
  echo "== old"; TSRL_LIB_PATH=variants/libtsrl_pl0.so timeout -k 10 200 $B || exit $?
  echo "== pair"; timeout -k 10 200 $B || exit $?
done
