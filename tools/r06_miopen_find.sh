#!/bin/bash
# (--conv-benchmark was a temporary bench.py flag for this A/B, removed after it measured no gain)
# Round-6 A/B on the config-5 bench: MIOpen immediate mode (default) vs find mode
# (--conv-benchmark on), two rounds, one box; then the find-mode profile's top kernels.
export TMPDIR=/tmp
for r in 1 2; do
  for m in off on; do
    echo "== conv-benchmark $m"; timeout -k 10 400 python3 bench.py --workload atari --steps 3 --warmup 2 --conv-benchmark $m 2>&1 | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']), round(d['ms_per_step'],1), d['config']['collect_s'], d['config']['update_s'])" || exit $?
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/fprof -o run -- python3 bench.py --workload atari --steps 2 --warmup 2 --conv-benchmark on > /dev/null 2>&1 || exit $?
python3 tools/rocpd_top.py /tmp/fprof/run_results.db 25 --last-ms 650 | cut -c1-150
rm -rf /tmp/fprof
