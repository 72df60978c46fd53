#!/bin/bash
# Round-5 A/B of the learn-side changes in mlp.hip (slab reductions with 16 lane groups; the
# eval tail's layer-1 tiles loaded one net ahead) against the previous mlp.hip
# (variants/libtsrl_old.so): parity of the new form, kernel times of both (rocprofv3, last
# iteration), then the update time alternating the two builds.
export TMPDIR=/tmp
T="python -u -m pytest -q -x -rf --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu"
B="python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline"
prof() {  # name lib
  TSRL_LIB_PATH=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$1 -o run -- $B > gpurun_out/prof_$1.log 2>&1 && python3 tools/rocpd_top.py gpurun_out/prof_$1/run_results.db 14 --last-ms 400 > gpurun_out/top_$1.txt && rm -rf gpurun_out/prof_$1
}
export -f prof
export B
tools/gpu_run.sh \
  "t_ev:600:$T tests/test_gpu_mlp.py tests/test_gpu_ppo.py tests/test_gpu_wide.py tests/test_gpu_rollout.py tests/test_gpu_fullsize.py tests/test_gpu_trainer.py" \
  "p_main:300:prof main ''" \
  "p_old:300:prof old variants/libtsrl_old.so" \
  "ab:900:for v in main old main old; do echo == \$v; if [ \$v = main ]; then L=; else L=variants/libtsrl_\$v.so; fi; TSRL_LIB_PATH=\$L timeout -k 10 150 $B 2>&1 | grep -E '^# iter' || exit 3; done" \
  "$@"
