#!/bin/bash
# Round-5 pipelined exact obs_rms, second A/B: the statistics kernel's XCD-aware column
# order (xcd), a 2048-row span (span2k: 20 KB LDS, two statistics fit beside a step
# workgroup), both (span2kxcd); one or two statistics branches.  Each variant's statistics
# are first checked bitwise against NumPy (tests/test_gpu_xpipe.py -k numpy).
export TMPDIR=/tmp
T="python -u -m pytest -q -x -rf --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu"
B="python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --exact-obs-rms"
run() {  # variant branches
  if [ $1 = main ]; then unset TSRL_LIB_PATH; else export TSRL_LIB_PATH=variants/libtsrl_$1.so; fi
  echo "== $1 branches $2"
  timeout -k 10 120 $B --exact-branches $2 | grep -E '^# iter 2|"value"' | sed 's/"roofline.*//'
}
tools/gpu_run.sh \
  "t_v:300:for v in xcd span2k span2kxcd; do TSRL_LIB_PATH=variants/libtsrl_\$v.so $T tests/test_gpu_xpipe.py -k numpy || exit \$?; done && TSRL_LIB_PATH=variants/libtsrl_span2kxcd.so $T tests/test_gpu_xpipe.py -k serial" \
  "ab:900:run main 1 && run main 2 && run xcd 1 && run xcd 2 && run span2k 1 && run span2k 2 && run span2kxcd 1 && run span2kxcd 2" \
  "$@"
