#!/bin/bash
# Round-5 A/B of the DMA-pipelined GAE row kernel (gae_rows_dma_kernel, default) against the
# staged one-row-per-workgroup kernel (TSRL_GAE_NODMA=1): parity, HIP-event times of the
# stand-alone launch loop (rew_norm and plain), rocprof kernel durations, then the bench line.
export TMPDIR=/tmp
T="python -u -m pytest -q -x -rf --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu"
G="python tools/gae_kernel_bench.py"
tools/gpu_run.sh \
  "t_gae:400:$T tests/test_gpu_gae.py tests/test_gpu_rollout.py tests/test_gpu_fullsize.py tests/test_gpu_wide.py" \
  "ab:400:for v in dma nodma dma nodma; do echo == \$v; if [ \$v = nodma ]; then export TSRL_GAE_NODMA=1; else unset TSRL_GAE_NODMA; fi; timeout -k 10 60 $G || exit 3; MODE=plain timeout -k 10 60 $G || exit 3; done" \
  "p_dma:200:ITERS=20 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pg_dma -o run -- $G && python3 tools/rocpd_top.py gpurun_out/pg_dma/run_results.db 4 > gpurun_out/gtop_dma.txt && rm -rf gpurun_out/pg_dma" \
  "p_nodma:200:TSRL_GAE_NODMA=1 ITERS=20 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pg_nodma -o run -- $G && python3 tools/rocpd_top.py gpurun_out/pg_nodma/run_results.db 4 > gpurun_out/gtop_nodma.txt && rm -rf gpurun_out/pg_nodma" \
  "bench:300:python3 bench.py --no-cpu-baseline" \
  "$@"
