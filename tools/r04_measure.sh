#!/bin/bash
# Round-4 measurement pass (one GPU call): GPU tests, smoke, the headline bench as the driver
# runs it, the other configs, the N>1 self-report rehearsal, rocprof kernel stats of the
# default and the exact-obs_rms bench (summaries go to profiles/ by hand).
export TMPDIR=/tmp
tools/gpu_run.sh \
  "tests:700:python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "smoke:120:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python -u bench.py" \
  "bench_exact:300:python -u bench.py --exact-obs-rms --no-cpu-baseline" \
  "bench_cpl:300:python -u bench.py --act-coef 0.05 --no-cpu-baseline" \
  "bench_small:200:python -u bench.py --workload small --no-cpu-baseline --steps 20" \
  "bench_forcedp:300:python -u -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --force-dp --no-cpu-baseline" \
  "prof:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --no-cpu-baseline" \
  "prof_exact:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_exact -o run -- python3 bench.py --exact-obs-rms --no-cpu-baseline --steps 1 --warmup 1" \
  "bench_atari:400:python -u bench.py --workload atari --steps 3" \
  "bench_cartpole:300:python -u bench.py --workload cartpole --steps 3"
