#!/bin/bash
# Round-5 check: is the GAE launch inside bench.py slowed by the permutation work that the
# side (plan) stream runs beside it?  The bench line's GAE launch times with the reference
# permutation stream (plan stream) and with --perm device (current stream, no side stream).
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline"
tools/gpu_run.sh \
  "ovl:500:for p in numpy device numpy device; do echo == \$p; timeout -k 10 150 $B --perm \$p 2>&1 | grep -E '^\{' | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d[\"roofline\"]; print(round(d[\"value\"]/1e6,2), \"M\", r[\"launch_us_each\"], round(r[\"frac\"],3), round(d[\"config\"][\"update_s\"]*1e3,1))' || exit 3; done" \
  "$@"
