#!/bin/bash
# Round-5 check: config 5 (Atari, conv trunk on MIOpen) with the learn epochs graph-captured
# (--graph-learn on) vs the default (conv trunks eager).
export TMPDIR=/tmp
B="python3 bench.py --workload atari --steps 3 --warmup 2 --no-cpu-baseline"
tools/gpu_run.sh \
  "ab:900:for v in auto on auto on; do echo == \$v; timeout -k 10 200 $B --graph-learn \$v > gpurun_out/a_\$v.log 2>&1 || exit 3; grep -E '^# iter 2|Warn|warn' gpurun_out/a_\$v.log | cut -c1-200; grep -E '^\{' gpurun_out/a_\$v.log | cut -c1-160; done" \
  "$@"
