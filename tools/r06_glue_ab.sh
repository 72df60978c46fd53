#!/bin/bash
# Round-6 A/B: config-5 glue cuts (first: flat Adam slots keep channels_last, the FC bias gradient as a
# HIP column sum, the FC weight gradient added straight into .grad, the Categorical loss's
# seed / zero fill / scaling passes skipped) -- this tree vs variants/oldtree (the previous
# commit's Python package, same libtsrl.so): the affected GPU tests on this tree, then the
# config-5 bench line twice interleaved.
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_atari.py tests/test_gpu_cartpole.py tests/test_gpu_ppo_discrete.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider 2>&1 | tail -4 || exit $?
for r in 1 2; do
  echo "== old"; timeout -k 10 300 python3 variants/oldtree/bench.py --workload atari --steps 3 --warmup 2 --no-cpu-baseline 2>&1 | grep -E '^# iter 2|^\{' | cut -c1-200 || exit $?
  echo "== new"; timeout -k 10 300 python3 bench.py --workload atari --steps 3 --warmup 2 --no-cpu-baseline 2>&1 | grep -E '^# iter 2|^\{' | cut -c1-200 || exit $?
done
