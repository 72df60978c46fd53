#!/bin/bash
# Round-6 A/B (TSRL_EVAL_CHUNK was a temporary override of FusedMLP.EVAL_CHUNK, since removed):
# process_fn evaluation chunk of the fused MLP (rows; the layer-1
# activations of a chunk, 512 B per row, reuse one buffer): 2M (1 GB, past the 256 MB
# Infinity Cache) vs 512k vs 256k rows, headline bench, two rounds, one box.
for r in 1 2; do
  for c in 2097152 524288 262144; do
    echo "== chunk $c"; TSRL_EVAL_CHUNK=$c timeout -k 10 300 python3 bench.py --no-cpu-baseline 2>&1 | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,3), round(d['ms_per_step'],2), round(d['config']['collect_s']*1e3,2), round(d['config']['update_s']*1e3,2))" || exit $?
  done
done
