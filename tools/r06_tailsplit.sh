#!/bin/bash
# Round-6 A/B: the headline's actor and critic tail kernels on two streams side by side at the
# full 262144-row minibatch (TSRL_TAIL_SPLIT_ROWS=1048576) vs one after the other (default),
# driver-form bench line twice interleaved.
for r in 1 2; do
  echo "== seq"; timeout -k 10 300 python3 bench.py --no-cpu-baseline > /tmp/b.log 2>&1 || exit $?; grep -E '^# iter 2' /tmp/b.log; grep -o '"value": [0-9.]*' /tmp/b.log
  echo "== split"; TSRL_TAIL_SPLIT_ROWS=1048576 timeout -k 10 300 python3 bench.py --no-cpu-baseline > /tmp/b.log 2>&1 || exit $?; grep -E '^# iter 2' /tmp/b.log; grep -o '"value": [0-9.]*' /tmp/b.log
done
