#!/bin/bash
# Round-6: the lane-contiguous H1 fragment layout (x6.h frag_off4) -- every GPU test, the
# layer-1 / minibatch / eval timings, then the headline bench.
export TMPDIR=/tmp
tools/gpu_run.sh \
  "tests:1200:python -u -m pytest tests -m gpu -q -rf --timeout 600 --timeout-method thread -p no:cacheprovider" \
  "kern:300:for i in 1 2; do python3 tools/mlp_kernel_bench.py --ld 384 --iters 30; done" \
  "bench:300:python -u bench.py --no-cpu-baseline" \
  "$@"
