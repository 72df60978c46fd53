#!/bin/bash
# Round-6 parity + measurement call: the full-length obs_rms reference test (both modes) and
# the whole-update reference test, then the three collect forms from ONE box (headline,
# action-coupled env, exact obs_rms) with the coupled env's run-to-run spread, then the
# collect step's counters on the shipped <3,false,false> instantiation (FETCH / WRITE / L2
# hit-miss, one pass each).
export TMPDIR=/tmp
P="timeout -s KILL 120 rocprofv3"
S="python3 tools/pmc_summary.py"
CB="python3 tools/collect_step_bench.py --steps 64 --reps 1"
tools/gpu_run.sh \
  "par:900:python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_update_full.py -v -rf --timeout 600 --timeout-method thread -p no:cacheprovider -s" \
  "bench:300:python -u bench.py" \
  "bench_coupled:300:python -u bench.py --act-coef 0.05 --no-cpu-baseline" \
  "bench_exact:300:python -u bench.py --exact-obs-rms --no-cpu-baseline" \
  "spread:300:python -u tools/coupled_spread.py" \
  "pmc_cf:150:$P --pmc FETCH_SIZE -d gpurun_out/pmc_cf -o run -- $CB && $S gpurun_out/pmc_cf/run_results.db collect_box > gpurun_out/pmc_cf.txt && rm -rf gpurun_out/pmc_cf" \
  "pmc_cw:150:$P --pmc WRITE_SIZE -d gpurun_out/pmc_cw -o run -- $CB && $S gpurun_out/pmc_cw/run_results.db collect_box > gpurun_out/pmc_cw.txt && rm -rf gpurun_out/pmc_cw" \
  "pmc_ch:150:$P --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_ch -o run -- $CB && $S gpurun_out/pmc_ch/run_results.db collect_box > gpurun_out/pmc_ch.txt && rm -rf gpurun_out/pmc_ch" \
  "$@"
