#!/bin/bash
# Round-5 A/B of the four default-off variants of round 4: correctness of
# each variant build on the collect / rollout / mlp tests, then the collect-step and dW1 A/B.
export TMPDIR=/tmp
T="python -u -m pytest -q -x -rf --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu"
tools/gpu_run.sh \
  "t_main:300:$T tests/test_gpu_padded.py tests/test_gpu_optim.py tests/test_gpu_stack.py" \
  "t_ek:300:TSRL_LIB_PATH=variants/libtsrl_ek.so $T tests/test_gpu_collect_step.py tests/test_gpu_rollout.py" \
  "t_oc:300:TSRL_LIB_PATH=variants/libtsrl_oc.so $T tests/test_gpu_collect_step.py tests/test_gpu_rollout.py" \
  "t_ns:300:TSRL_LIB_PATH=variants/libtsrl_ns.so $T tests/test_gpu_collect_step.py tests/test_gpu_rollout.py" \
  "t_all3:300:TSRL_LIB_PATH=variants/libtsrl_all3.so $T tests/test_gpu_collect_step.py tests/test_gpu_rollout.py" \
  "t_dwfull:300:TSRL_LIB_PATH=variants/libtsrl_dwfull.so $T tests/test_gpu_mlp.py" \
  "ab_collect:600:tools/collect_ab.sh ek oc ns all3 && tools/collect_ab.sh all3 main" \
  "ab_dw:400:tools/dw_ab.sh dwfull"
