#!/bin/bash
# Round-6 call 3: the two reference-parity tests after the assertion rework, then the l1_ring
# diagnostic variants and one SQ counter pass on the shipped l1_ring_kernel.
export TMPDIR=/tmp
P="timeout -s KILL 90 rocprofv3"
tools/gpu_run.sh \
  "par:900:python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_update_full.py -v -rf --timeout 600 --timeout-method thread -p no:cacheprovider -s" \
  "l1diag:500:tools/r06_l1diag.sh" \
  "pmc_l1:120:$P --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/pmc_l1 -o run -- python3 tools/mlp_kernel_bench.py --only l1_fwd_x6 --ld 384 --iters 5 && python3 tools/pmc_summary.py gpurun_out/pmc_l1/run_results.db l1_ring > gpurun_out/pmc_l1.txt && rm -rf gpurun_out/pmc_l1" \
  "$@"
