#!/bin/bash
# Collect-step A/B at the headline shape: the in-tree library, then each variant named on the
# command line (variants/libtsrl_<name>.so from tools/build_variant.sh, e.g. a
# -D... build of collect.hip, e.g. the round-5 A/B of tools/r05_ab.sh).
set -o pipefail
for v in main "$@"; do
  if [ $v = main ]; then unset TSRL_LIB_PATH; else export TSRL_LIB_PATH=variants/libtsrl_$v.so; fi
  echo "== $v"
  timeout -k 10 150 python tools/collect_step_bench.py --steps 256 --reps 3 || exit $?
done
