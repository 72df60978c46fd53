#!/bin/bash
# Round-5 A/B: the layer-1 and dW1 products with the 24 MFMAs of a 16-k step interleaved over
# the four accumulators (variants il4 = mlp_x6.hip -DL1_IL4, dwil4 = mlp.hip -DDW_IL4) against
# the in-tree pair-interleaved / per-tile order: parity of each variant, then kernel times.
export TMPDIR=/tmp
T="python -u -m pytest -q -x -rf --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu"
K="python tools/mlp_kernel_bench.py --iters 20"
tools/gpu_run.sh \
  "t_il4:300:TSRL_LIB_PATH=variants/libtsrl_il4.so $T tests/test_gpu_mlp.py tests/test_gpu_ppo.py" \
  "t_dwil4:300:TSRL_LIB_PATH=variants/libtsrl_dwil4.so $T tests/test_gpu_mlp.py tests/test_gpu_ppo.py" \
  "ab:900:for v in main il4 dwil4 main il4 dwil4; do echo == \$v; if [ \$v = main ]; then L=; else L=variants/libtsrl_\$v.so; fi; TSRL_LIB_PATH=\$L timeout -k 10 120 $K --only l1_fwd_x6 || exit 3; TSRL_LIB_PATH=\$L timeout -k 10 120 $K --only dw || exit 3; TSRL_LIB_PATH=\$L timeout -k 10 120 $K --only minibatch || exit 3; done" \
  "$@"
