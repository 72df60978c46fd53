#!/bin/bash
# Round-3 measurement pass (one GPU call): GPU tests, smoke, headline bench, rocprof kernel
# stats of the bench (summaries go to profiles/ by hand).
export TMPDIR=/tmp
tools/gpu_run.sh \
  "tests:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python -u bench.py" \
  "prof:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 3"
