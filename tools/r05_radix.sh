#!/bin/bash
# Round-5 hand-written LSD radix sort in the permutation resolution (csrc/perm.hip, replacing
# hipcub::DeviceRadixSort): bit-exactness vs NumPy's permutation and the learn goldens, then the
# bench line and a kernel profile of the permutation kernels.
export TMPDIR=/tmp
T="python -u -m pytest -q -x -rf --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu"
tools/gpu_run.sh \
  "t_perm:600:$T tests/test_gpu_perm.py tests/test_gpu_ppo.py tests/test_gpu_trainer.py tests/test_gpu_a_dist.py" \
  "bench:300:python3 bench.py --no-cpu-baseline" \
  "prof:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --no-cpu-baseline && python3 tools/rocpd_top.py gpurun_out/prof/run_results.db 40 > gpurun_out/kernel_top.txt && rm -rf gpurun_out/prof" \
  "$@"
