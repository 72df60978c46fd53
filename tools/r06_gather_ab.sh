#!/bin/bash
# Round-6 A/B: eager Categorical minibatches hand autograd's gradients over (.grad = None before
# (reused for the follow-up: the FC weight gradient written into its released flat slot)
# backward, one multi-tensor copy into the flat bucket after: FlatAdam.release_grads /
# gather_grads) vs the zero-filled bucket + per-parameter adds (variants/oldtree = the previous
# commit's Python package, same libtsrl.so): the affected GPU tests, then config 5 twice interleaved.
timeout -k 10 600 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_atari.py tests/test_gpu_cartpole.py tests/test_gpu_ppo_discrete.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider 2>&1 | tail -4 || exit $?
for r in 1 2; do
  echo "== old"; timeout -k 10 300 python3 variants/oldtree/bench.py --workload atari --steps 3 --warmup 2 --no-cpu-baseline > /tmp/b.log 2>&1 || exit $?; grep -E '^# iter 2|^\{' /tmp/b.log | cut -c1-200
  echo "== new"; timeout -k 10 300 python3 bench.py --workload atari --steps 3 --warmup 2 --no-cpu-baseline > /tmp/b.log 2>&1 || exit $?; grep -E '^# iter 2|^\{' /tmp/b.log | cut -c1-200
done
timeout -k 10 400 python3 tools/atari_torchprof.py --top 16 > /tmp/tp.txt 2>&1 || exit $?; grep -v "^/opt\|Warn\|warn" /tmp/tp.txt
