#!/bin/bash
# Round-5 measurement pass (one GPU call): GPU tests, smoke, the headline bench as the driver
# runs it, rocprof kernel stats of the bench (summarised on the box by tools/rocpd_top.py; the
# summaries go to profiles/ by hand).
# Usage: tools/r05_measure.sh [extra gpu_run.sh steps...]
export TMPDIR=/tmp
tools/gpu_run.sh \
  "tests:900:python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider -s" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python -u bench.py" \
  "prof:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --no-cpu-baseline && python3 tools/rocpd_top.py gpurun_out/prof/run_results.db > gpurun_out/kernel_top.txt && rm -rf gpurun_out/prof" \
  "$@"
