#!/bin/bash
# Round-6 A/B: process_fn's evaluation fused into the layer-1 ring (tsrl_ppo_eval_fused,
# default) vs tsrl_mlp_l1_fwd_x6 + tsrl_ppo_eval per 2M-row chunk (TSRL_EVAL_FUSED=0):
# MLP / process_fn / full-size tests first, then the headline bench twice interleaved and a
# rocprof kernel summary of the fused form.
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_wide.py tests/test_gpu_ppo.py tests/test_gpu_fullsize.py -q -rf --timeout 600 --timeout-method thread -p no:cacheprovider 2>&1 | tail -4 || exit $?
for r in 1 2; do
  for f in 0 1; do
    echo "== fused $f"; TSRL_EVAL_FUSED=$f timeout -k 10 300 python3 bench.py --no-cpu-baseline 2>&1 | grep '^{' | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,3), round(d['ms_per_step'],2), round(d['config']['collect_s']*1e3,2), round(d['config']['update_s']*1e3,2))" || exit $?
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/fprof -o run -- python3 bench.py --steps 3 --no-cpu-baseline > /dev/null 2>&1 || exit $?
python3 tools/rocpd_top.py /tmp/fprof/run_results.db 14 | cut -c1-170
rm -rf /tmp/fprof
