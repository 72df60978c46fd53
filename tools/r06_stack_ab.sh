#!/bin/bash
# Round-6 A/B: frame-stack gather with batched 16-byte loads (this build) vs one load-store round
# (STACK_BATCHED was removed after the measurement -- rejected)
# trip per piece (variants/libtsrl_sg0.so = -DSTACK_BATCHED=0): buffer / atari GPU tests on this
# build, then sample(0) timing + checksum of the stacked obs, twice interleaved.
timeout -k 10 600 python -u -m pytest tests/test_gpu_atari.py tests/test_gpu_padded.py tests/test_gpu_stack.py tests/test_gpu_fullsize.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2 || exit $?
for r in 1 2; do
  echo "== old"; TSRL_LIB_PATH=variants/libtsrl_sg0.so timeout -k 10 200 python3 tools/stack_gather_bench.py > /tmp/s.log 2>&1 || exit $?; grep -v amdgpu /tmp/s.log
  echo "== new"; timeout -k 10 200 python3 tools/stack_gather_bench.py > /tmp/s.log 2>&1 || exit $?; grep -v amdgpu /tmp/s.log
done
