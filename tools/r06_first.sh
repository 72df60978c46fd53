#!/bin/bash
# Round-6 first GPU pass: the new whole-update parity test + the data-parallel / optimiser
# tests touched by the shard-table and clip_adam changes, then the GAE PMC passes on the
# changed gae.hip (host-side only change; bench.py matches the record by source sha).
export TMPDIR=/tmp
P="timeout -s KILL 120 rocprofv3"
tools/gpu_run.sh \
  "upd:600:python -u -m pytest tests/test_gpu_update_full.py tests/test_gpu_optim.py tests/test_gpu_a_dist.py tests/test_gpu_a0_nccl.py -v -rf --timeout 300 --timeout-method thread -p no:cacheprovider -s" \
  "pmc_gf:150:$P --pmc FETCH_SIZE -d gpurun_out/pmc_gf -o run -- python3 tools/gae_kernel_bench.py" \
  "pmc_gw:150:$P --pmc WRITE_SIZE -d gpurun_out/pmc_gw -o run -- python3 tools/gae_kernel_bench.py" \
  "pmc_gj:60:python3 tools/pmc_gae.py --db gpurun_out/pmc_gf/run_results.db gpurun_out/pmc_gw/run_results.db gpurun_out/r06_gae_pmc.json && rm -rf gpurun_out/pmc_gf gpurun_out/pmc_gw" \
  "$@"
