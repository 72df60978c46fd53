#!/bin/bash
# Round-6 probe: config 5 with MIOpen's NHWC implicit-GEMM asm solvers (GTC XDLOPS) disabled one
# at a time (MIOpen then falls back to its next applicable solver), vs the default.
B="python3 bench.py --workload atari --steps 3 --warmup 2 --no-cpu-baseline"
run() { echo "== $1"; env $2 timeout -k 10 400 $B > /tmp/b.log 2>&1 || { echo "rc=$?"; tail -3 /tmp/b.log; return 0; }; grep -E '^# iter 2' /tmp/b.log; grep -o '"value": [0-9.]*' /tmp/b.log; }
run default ""
run bwd_off "MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0"
run wrw_off "MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0"
run fwd_off "MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0"
run default ""
