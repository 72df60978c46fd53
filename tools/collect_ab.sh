#!/bin/bash
# Collect-step store-form A/B (COLLECT_ROW_STORE variants) at the headline shape.
set -o pipefail
for v in main crs1 crs2; do
  if [ $v = main ]; then unset TSRL_LIB_PATH; else export TSRL_LIB_PATH=variants/libtsrl_$v.so; fi
  echo "== $v"
  timeout -k 10 150 python tools/collect_step_bench.py --steps 256 --reps 3 || exit $?
done
