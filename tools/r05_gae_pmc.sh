#!/bin/bash
# Round-5 HBM counter passes of the GAE kernel at the bench shape (the roofline the bench line
# names): FETCH_SIZE and WRITE_SIZE in separate rocprofv3 runs of tools/gae_kernel_bench.py,
# folded on the box into profiles-ready JSON (tools/pmc_gae.py --db, which records the
# gae.hip sha256), then the databases are deleted so gpurun_out/ stays small.
export TMPDIR=/tmp
P="timeout -s KILL 120 rocprofv3"
tools/gpu_run.sh \
  "pmc_gf:150:$P --pmc FETCH_SIZE -d gpurun_out/pmc_gf -o run -- python3 tools/gae_kernel_bench.py" \
  "pmc_gw:150:$P --pmc WRITE_SIZE -d gpurun_out/pmc_gw -o run -- python3 tools/gae_kernel_bench.py" \
  "pmc_gj:60:python3 tools/pmc_gae.py --db gpurun_out/pmc_gf/run_results.db gpurun_out/pmc_gw/run_results.db gpurun_out/r05_gae_pmc.json && rm -rf gpurun_out/pmc_gf gpurun_out/pmc_gw" \
  "$@"
