#!/bin/bash
# Round-6 A/B on the config-5 bench: this build vs variants/libtsrl_f.so (dqn_conv.hip of
# commit facb01d: single-buffer conv1 forward, one class per conv2-gradient workgroup), two
# rounds, one box; then the kernels of both.
for r in 1 2; do
  echo "== facb01d"; TSRL_LIB_PATH=variants/libtsrl_f.so timeout -k 10 300 python3 bench.py --workload atari --steps 3 --warmup 2 2>&1 | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],1), d['config']['collect_s'], d['config']['update_s'])" || exit $?
  echo "== head"; timeout -k 10 300 python3 bench.py --workload atari --steps 3 --warmup 2 2>&1 | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],1), d['config']['collect_s'], d['config']['update_s'])" || exit $?
done
echo "== facb01d kernels"; TSRL_LIB_PATH=variants/libtsrl_f.so timeout -k 10 120 python3 tools/atari_kernel_ab.py || exit $?
echo "== head kernels"; timeout -k 10 120 python3 tools/atari_kernel_ab.py || exit $?
