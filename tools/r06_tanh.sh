#!/bin/bash
# Round-6 A/B: tanh_nb's large-|x| half from v_exp_f32 (2^(2|x| log2 e)) instead of expf's
# range-reduced exp (variants/libtsrl_texp2.so: mlp.hip + mlp_x6.hip with -DTANH_EXP2), kernel
# timings interleaved twice, then the MLP parity tests on the variant.
B="python3 tools/mlp_kernel_bench.py --ld 384 --iters 30"
for r in 1 2; do
  echo "== base"; timeout -k 10 120 $B || exit $?
  echo "== exp2"; TSRL_LIB_PATH=variants/libtsrl_texp2.so timeout -k 10 120 $B || exit $?
done
echo "== tests (exp2)"
TSRL_LIB_PATH=variants/libtsrl_texp2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_ppo.py tests/test_gpu_wide.py tests/test_gpu_rollout.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider 2>&1 | tail -4
