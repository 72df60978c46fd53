#!/bin/bash
# Round-5 exact obs_rms defaults (depth 5, two steps per statistics launch): the exact-mode
# parity tests, then the exact-mode bench and a default-mode bench in the same call.
export TMPDIR=/tmp
T="python -u -m pytest -q -x -rf --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu"
tools/gpu_run.sh \
  "tx:600:$T tests/test_gpu_xpipe.py tests/test_gpu_wide.py tests/test_gpu_rollout.py" \
  "bx:300:python3 bench.py --exact-obs-rms" \
  "bd:300:python3 bench.py" \
  "$@"
