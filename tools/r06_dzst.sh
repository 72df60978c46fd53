#!/bin/bash
# Round-6: the tails' dZ1 tile stored through the wave's LDS scratch as whole-row runs -- MLP /
# PPO parity tests, then tail / minibatch timings (this build), twice.
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_ppo.py tests/test_gpu_wide.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider 2>&1 | tail -3 || exit $?
for r in 1 2; do timeout -k 10 200 python3 tools/mlp_kernel_bench.py --ld 384 --iters 30 || exit $?; done
