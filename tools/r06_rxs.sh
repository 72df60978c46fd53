#!/bin/bash
# (the build flags this recipe names were removed after the measurement; the recipe documents
# how the committed log was produced -- rebuild the variants from the commit it cites to rerun)
# Round-6 probe: the layer-1 ring with a 2-stage X ring (X issued one chunk ahead;
# variants/libtsrl_x2.so = -DL1_RXS=2) vs the shipped 3 stages -- would a fused process_fn
# evaluation (layer-2 images beside the ring) fit?  MLP tests on the variant, then the kernel
# bench twice interleaved (gathered minibatch rows and contiguous 2M-row evaluation).
TSRL_LIB_PATH=variants/libtsrl_x2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_wide.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2 || exit $?
B="python3 tools/mlp_kernel_bench.py --ld 384 --iters 30"
for r in 1 2; do
  echo "== rxs3"; timeout -k 10 200 $B | grep -E "l1_fwd|eval" || exit $?
  echo "== rxs2"; TSRL_LIB_PATH=variants/libtsrl_x2.so timeout -k 10 200 $B | grep -E "l1_fwd|eval" || exit $?
done
