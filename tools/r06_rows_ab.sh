#!/bin/bash
# Round-6 A/B: config-5 minibatches read from the whole batch in place by the uint8 trunk
# kernels (default) vs gathered into a minibatch copy first (TSRL_TRUNK_ROWS=0); the atari
# GPU tests first, then the config-5 bench twice interleaved.
timeout -k 10 400 python -u -m pytest tests/test_gpu_atari.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2 || exit $?
for r in 1 2; do
  for f in 0 1; do
    echo "== rows $f"; TSRL_TRUNK_ROWS=$f timeout -k 10 300 python3 bench.py --workload atari --steps 3 --warmup 2 2>&1 | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],1), round(d['config']['collect_s']*1e3,1), round(d['config']['update_s']*1e3,1))" || exit $?
  done
done
