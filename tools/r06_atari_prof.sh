#!/bin/bash
# Round 6: config-5 (atari) steady-state profile + per-layer timings of the trunk.
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/atari_layer_bench.py --rows 8192 --iters 10 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/aprof -o run -- python3 bench.py --workload atari --steps 2 --warmup 2 > gpurun_out/atari_bench.log 2>&1 || exit $?
db=$(find /tmp/aprof -name '*results.db' | head -1)
python3 tools/rocpd_top.py "$db" 40 --last-ms 700 > gpurun_out/atari_top.txt
tail -1 gpurun_out/atari_bench.log >> gpurun_out/atari_top.txt
rm -rf /tmp/aprof
