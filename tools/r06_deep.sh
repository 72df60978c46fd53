#!/bin/bash
# Round-6 A/B of l1_deep_kernel (TSRL_L1_DEEP=1) against l1_ring_kernel: the MLP / PPO parity
# tests with the deep kernel, then the layer-1 timing (gathered rows pitch 384, and contiguous
# rows as in process_fn), each form twice, interleaved.
B="python3 tools/mlp_kernel_bench.py --only l1_fwd_x6 --ld 384 --iters 30"
echo "== tests (deep)"
TSRL_L1_DEEP=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_ppo.py -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider 2>&1 | tail -5 || exit $?
for r in 1 2; do
  echo "== ring"; timeout -k 10 120 $B || exit $?
  echo "== deep"; TSRL_L1_DEEP=1 timeout -k 10 120 $B || exit $?
  echo "== ring contig"; timeout -k 10 120 $B --contig || exit $?
  echo "== deep contig"; TSRL_L1_DEEP=1 timeout -k 10 120 $B --contig || exit $?
done
