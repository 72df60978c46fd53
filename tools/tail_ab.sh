#!/bin/bash
# Tail-kernel A/B at the benchmark shape: the in-tree library, then each variant named on the
# command line (variants/libtsrl_<name>.so from tools/build_variant.sh mlp.hip -D...).
# A TAIL_TRACE=1 variant is reported per phase instead: tools/tail_ab.sh trace:<name>.
set -o pipefail
for v in main "$@"; do
  unset TSRL_LIB_PATH
  case $v in
    main) ;;
    trace:*) export TSRL_LIB_PATH=variants/libtsrl_${v#trace:}.so
             timeout -k 10 120 python tools/mlp_kernel_bench.py --tail-trace 4 || exit $?; continue ;;
    *) export TSRL_LIB_PATH=variants/libtsrl_$v.so ;;
  esac
  echo "== $v"
  timeout -k 10 120 python tools/mlp_kernel_bench.py --iters 20 --only tail || exit $?
done
