#!/bin/bash
# Round-5 pipelined exact obs_rms (csrc/collect.hip E): the statistics kernel alone, parity
# (the new tests, the exact reference goldens, the wide and collect-step tests), then the
# exact-mode bench pipelined (depth 2, 1, 3) vs serial, the default bench, and a kernel trace
# of the pipelined form.
export TMPDIR=/tmp
T="python -u -m pytest -q -x -rf --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu"
B="python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline"
tools/gpu_run.sh \
  "xs:200:python tools/xstats_bench.py" \
  "t_x:400:$T tests/test_gpu_xpipe.py tests/test_gpu_rollout.py tests/test_gpu_wide.py tests/test_gpu_collect_step.py" \
  "b_xpipe:300:$B --exact-obs-rms" \
  "b_x1:300:$B --exact-obs-rms --exact-pipeline 1" \
  "b_x3:300:$B --exact-obs-rms --exact-pipeline 3" \
  "b_serial:300:$B --exact-obs-rms --exact-pipeline 0" \
  "b_default:300:$B" \
  "p_xpipe:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_x -o run -- $B --exact-obs-rms && python3 tools/rocpd_top.py gpurun_out/prof_x/run_results.db > gpurun_out/xpipe_top.txt && rm -rf gpurun_out/prof_x" \
  "$@"
