import sqlite3
from collections import defaultdict
"""Round-4 form: python tools/pmc_learn.py [out.txt] after the two passes
    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o run -- python3 tools/mlp_kernel_bench.py --only minibatch --ld 384
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o run -- python3 tools/mlp_kernel_bench.py --only minibatch --ld 384
"""
import sys

KEYS = {"l1_ring_kernel": ("l1_ring_kernel",),
        "ppo_tail_kernel<0>": ("ppo_tail_kernel<0>", "ppo_tail_kernelILi0E"),
        "ppo_tail_kernel<1>": ("ppo_tail_kernel<1>", "ppo_tail_kernelILi1E"),
        "dw_x6_kernel": ("dw_x6_kernel",), "tail_reduce_kernel": ("tail_reduce_kernel",),
        "dw_reduce_kernel": ("dw_reduce_kernel",), "clip_adam_kernel": ("clip_adam_kernel",)}


def load(db):
    c = sqlite3.connect(db)
    acc = defaultdict(list)
    for name, cn, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
        for k, pats in KEYS.items():
            if any(p in name for p in pats):
                acc[(k, cn)].append(v)
    return acc
f = load("gpurun_out/pmc_f/run_results.db"); w = load("gpurun_out/pmc_w/run_results.db")
B, D = 262144, 376
alg = {  # algorithmic HBM bytes per launch (read, write) at 262144 rows, D = 376, A = 17
    "l1_ring_kernel": (B * D * 4, B * 128 * 4),
    "ppo_tail_kernel<0>": (B * 64 * 4 + B * (17 + 2) * 4, B * 64 * 4),
    "ppo_tail_kernel<1>": (B * 64 * 4 + B * 2 * 4, B * 64 * 4),
    "dw_x6_kernel": (B * D * 4 + B * 128 * 4, 168 * 128 * 384 * 4),
    "tail_reduce_kernel": (256 * (2 * 64 * 64 + 2 * 64 + 32 * 64 + 32 + 64 + 4) * 4, 0),
    "dw_reduce_kernel": (168 * 128 * 384 * 4, 128 * 377 * 4),
    "clip_adam_kernel": (57763 * 4 * 4, 57763 * 3 * 4),
}
out_lines = []
_print = print


def print(*a, **k):  # noqa: A001 - tee the report
    s = " ".join(str(x) for x in a)
    out_lines.append(s)
    _print(s, **k)
print("# PMC HBM bytes per launch of one 262144-row PPO minibatch (tools/mlp_kernel_bench.py --only minibatch")
print("# --ld 384: random rows of the padded 384-float storage pitch, D=376, A=17), two rocprofv3 --pmc passes")
print("# (FETCH_SIZE; WRITE_SIZE), means over the dispatches.")
print("# FETCH_SIZE doubled (gfx950 tallies 64 B per 128-B read request, MI355X_MICROARCH.md HBM section);")
print("# algorithmic = bytes the kernel must move: gathered X rows, h1/dZ1 halves, per-row act/logp/adv/ret/v_s,")
print("# dW partial slabs (168 row splits x 128 x 384 f32).")
print(f"{'kernel':26s} {'read MB':>9s} {'alg MB':>8s} {'x':>6s} {'write MB':>9s} {'alg MB':>8s} {'x':>6s}")
tot_r = tot_w = 0
for k, (ar, aw) in alg.items():
    if not f[(k, "FETCH_SIZE")] or not w[(k, "WRITE_SIZE")]:
        continue
    r = 2 * 1024 * sum(f[(k, "FETCH_SIZE")]) / len(f[(k, "FETCH_SIZE")])
    wr = 1024 * sum(w[(k, "WRITE_SIZE")]) / len(w[(k, "WRITE_SIZE")])
    tot_r += r; tot_w += wr
    xr = f"{r/ar:6.2f}" if ar else "   -  "
    xw = f"{wr/aw:6.2f}" if aw else "   -  "
    print(f"{k:26s} {r/1e6:9.1f} {ar/1e6:8.1f} {xr} {wr/1e6:9.1f} {aw/1e6:8.1f} {xw}")
print(f"{'total (minibatch kernels)':26s} {tot_r/1e6:9.1f} {'':8s} {'':6s} {tot_w/1e6:9.1f}")
print(f"# HBM bytes per minibatch {(tot_r+tot_w)/1e9:.2f} GB; compulsory for a fused per-tile minibatch (X once + per-row")
print(f"# inputs, h1/dZ1 on chip): {(B*D*4 + B*21*4)/1e6:.0f} MB read")
print(f"# ratio to that compulsory read: {(tot_r + tot_w) / (B*D*4 + B*21*4):.2f}x")
if len(sys.argv) > 1:
    with open(sys.argv[1], "w") as fh:
        fh.write("\n".join(out_lines) + "\n")
