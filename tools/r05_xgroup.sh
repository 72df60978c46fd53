#!/bin/bash
# Round-5 pipelined exact obs_rms, grouped statistics launches (Collector.exact_group): parity
# (tests/test_gpu_xpipe.py), then collect times for depth / group / branches combinations.
export TMPDIR=/tmp
T="python -u -m pytest -q -x -rf --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu"
B="python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --exact-obs-rms"
run() {  # depth group branches
  echo "== depth $1 group $2 branches $3"
  timeout -k 10 120 $B --exact-pipeline $1 --exact-group $2 --exact-branches $3 2>&1 | grep -E '^# iter 2'
}
export -f run
export B
tools/gpu_run.sh \
  "ab:900:run 4 2 1 && run 5 2 1 && run 6 2 1 && run 5 2 2 && run 6 2 2 && run 4 2 1" \
  "$@"
