#!/bin/bash
# Round-6 measurement pass (one GPU call): every GPU test, smoke, the headline bench as the
# driver runs it plus the two other collect forms from the same box (action-coupled env,
# exact obs_rms), the coupled env's run-to-run spread, rocprof kernel stats of the bench, and
# the collect step's counters (FETCH / WRITE / L2 hit-miss, one pass each); config 5's bench line
# and steady-state kernel profile.
export TMPDIR=/tmp
P="timeout -s KILL 120 rocprofv3"
S="python3 tools/pmc_summary.py"
CB="python3 tools/collect_step_bench.py --steps 64 --reps 1"
tools/gpu_run.sh \
  "tests:1200:python -u -m pytest tests -m gpu -q -rf --timeout 600 --timeout-method thread -p no:cacheprovider -s" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python -u bench.py" \
  "bench_coupled:300:python -u bench.py --act-coef 0.05 --no-cpu-baseline" \
  "bench_exact:300:python -u bench.py --exact-obs-rms --no-cpu-baseline" \
  "spread:300:python -u tools/coupled_spread.py" \
  "prof:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --no-cpu-baseline && python3 tools/rocpd_top.py gpurun_out/prof/run_results.db > gpurun_out/kernel_top.txt && rm -rf gpurun_out/prof" \
  "bench_atari:300:python -u bench.py --workload atari --steps 3 --warmup 2" \
  "prof_atari:400:rocprofv3 --kernel-trace --stats -d /tmp/aprof -o run -- python3 bench.py --workload atari --steps 2 --warmup 2 --no-cpu-baseline > gpurun_out/prof_atari_bench.log 2>&1 && python3 tools/rocpd_top.py /tmp/aprof/run_results.db 40 --last-ms 650 > gpurun_out/atari_top.txt && rm -rf /tmp/aprof" \
  "pmc_cf:150:$P --pmc FETCH_SIZE -d gpurun_out/pmc_cf -o run -- $CB && $S gpurun_out/pmc_cf/run_results.db collect_box > gpurun_out/pmc_cf.txt && rm -rf gpurun_out/pmc_cf" \
  "pmc_cw:150:$P --pmc WRITE_SIZE -d gpurun_out/pmc_cw -o run -- $CB && $S gpurun_out/pmc_cw/run_results.db collect_box > gpurun_out/pmc_cw.txt && rm -rf gpurun_out/pmc_cw" \
  "pmc_ch:150:$P --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_ch -o run -- $CB && $S gpurun_out/pmc_ch/run_results.db collect_box > gpurun_out/pmc_ch.txt && rm -rf gpurun_out/pmc_ch" \
  "$@"
