#!/bin/bash
# Round-5 A/B: small minibatches (config 2's 2048 rows) with the actor's and the critic's tail
# kernels on two streams side by side (default) vs one stream (TSRL_TAIL_SPLIT=0): parity
# (learn goldens, graph-captured epochs), then config 2's update time.
export TMPDIR=/tmp
T="python -u -m pytest -q -x -rf --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu"
B="python3 bench.py --workload small --steps 3 --warmup 2 --no-cpu-baseline"
tools/gpu_run.sh \
  "t_split:600:$T tests/test_gpu_ppo.py tests/test_gpu_mlp.py tests/test_gpu_trainer.py tests/test_gpu_sched.py tests/test_gpu_padded.py" \
  "ab:700:for v in split one split one; do echo == \$v; if [ \$v = one ]; then export TSRL_TAIL_SPLIT=0; else unset TSRL_TAIL_SPLIT; fi; timeout -k 10 150 $B > gpurun_out/b_\$v.log 2>&1 || exit 3; grep -E '^# iter 2|^\{' gpurun_out/b_\$v.log | cut -c1-200; done" \
  "$@"
