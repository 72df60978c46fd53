#!/bin/bash
# Round-5 A/B of the slab reductions (tail_reduce / dw_reduce: 16 lane groups per block vs the
# round-4 form's 4, variants/libtsrl_ng4.so): learn-path parity on the new form, then the
# update time of the default bench, alternating the two builds.
export TMPDIR=/tmp
T="python -u -m pytest -q -x -rf --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu"
B="python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline"
tools/gpu_run.sh \
  "t_slab:600:$T tests/test_gpu_mlp.py tests/test_gpu_ppo.py tests/test_gpu_trainer.py tests/test_gpu_sched.py" \
  "ab:900:for v in main ng4 main ng4; do echo == \$v; if [ \$v = main ]; then L=; else L=variants/libtsrl_\$v.so; fi; TSRL_LIB_PATH=\$L timeout -k 10 150 $B 2>&1 | grep -E '^# iter' || exit 3; done" \
  "$@"
