#!/bin/bash
# Round 6: config-5 bench lines, this build vs variants/libtsrl_g.so (gathered trunk kernels),
# twice interleaved; then the conv kernels' A/B.
for r in 1 2; do
  echo "== gather"; TSRL_LIB_PATH=variants/libtsrl_g.so timeout -k 10 300 python3 bench.py --workload atari --steps 3 --warmup 2 2>&1 | tail -1 || exit $?
  echo "== lds"; timeout -k 10 300 python3 bench.py --workload atari --steps 3 --warmup 2 2>&1 | tail -1 || exit $?
done
timeout -k 10 120 python3 tools/atari_kernel_ab.py || exit $?
