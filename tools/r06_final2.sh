#!/bin/bash
# Round 6, second final-tree check (after the config-5 glue cuts and the gradient hand-over):
# every GPU test + smoke, the driver-form bench line, config 5's line.
tools/gpu_run.sh \
  "tests:900:python -u -m pytest tests -m gpu -q -rf --timeout 600 --timeout-method thread -p no:cacheprovider" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python -u bench.py" \
  "bench_atari:300:python -u bench.py --workload atari --steps 3 --warmup 2 --no-cpu-baseline" \
  "$@"
