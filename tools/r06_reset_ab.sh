#!/bin/bash
# Round-6 check: u8 resets written straight into the collector's current obs (no masked select
# pass); the u8 / frame-stack GPU tests, then the config-5 bench twice.
timeout -k 10 600 python -u -m pytest tests/test_gpu_atari.py tests/test_gpu_stack.py tests/test_gpu_rollout.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2 || exit $?
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --workload atari --steps 3 --warmup 2 2>&1 | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],1), round(d['config']['collect_s']*1e3,1), round(d['config']['update_s']*1e3,1))" || exit $?
done
