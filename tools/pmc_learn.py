import sqlite3
from collections import defaultdict
def load(db):
    c = sqlite3.connect(db)
    acc = defaultdict(list)
    for name, cn, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
        n = name.replace("tsrl::(anonymous namespace)::", "").split("(")[0]
        acc[(n, cn)].append(v)
    return acc
f = load("gpurun_out/pmc_f/run_results.db"); w = load("gpurun_out/pmc_w/run_results.db")
B, D = 262144, 376
alg = {  # algorithmic HBM bytes per launch (read, write) at 262144 rows, D = 376, A = 17
    "l1_fwd_x6_kernel": (B * D * 4, B * 128 * 4),
    "void ppo_tail_kernel<0>": (B * 64 * 4 + B * (17 + 2) * 4, B * 64 * 4),
    "void ppo_tail_kernel<1>": (B * 64 * 4 + B * 2 * 4, B * 64 * 4),
    "dw_x6_kernel": (B * D * 4 + B * 128 * 4, 168 * 128 * 384 * 4),
}
print("# PMC HBM bytes per launch of one 262144-row PPO minibatch (tools/mlp_kernel_bench.py --only minibatch,")
print("# random rows, D=376, A=17), two rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE), means over the dispatches.")
print("# FETCH_SIZE doubled (gfx950 tallies 64 B per 128-B read request, MI355X_MICROARCH.md HBM section);")
print("# algorithmic = bytes the kernel must move: gathered X rows, h1/dZ1 halves, per-row act/logp/adv/ret/v_s,")
print("# dW partial slabs (168 row splits x 128 x 384 f32).")
print(f"{'kernel':26s} {'read MB':>9s} {'alg MB':>8s} {'x':>6s} {'write MB':>9s} {'alg MB':>8s} {'x':>6s}")
tot_r = tot_w = 0
for k, (ar, aw) in alg.items():
    r = 2 * 1024 * sum(f[(k, "FETCH_SIZE")]) / len(f[(k, "FETCH_SIZE")])
    wr = 1024 * sum(w[(k, "WRITE_SIZE")]) / len(w[(k, "WRITE_SIZE")])
    tot_r += r; tot_w += wr
    print(f"{k:26s} {r/1e6:9.1f} {ar/1e6:8.1f} {r/ar:6.2f} {wr/1e6:9.1f} {aw/1e6:8.1f} {wr/aw:6.2f}")
print(f"{'total (4 main kernels)':26s} {tot_r/1e6:9.1f} {'':8s} {'':6s} {tot_w/1e6:9.1f}")
print(f"# HBM bytes per minibatch {(tot_r+tot_w)/1e9:.2f} GB; compulsory for a fused per-tile minibatch (X once + per-row")
print(f"# inputs, h1/dZ1 on chip): {(B*D*4 + B*21*4)/1e6:.0f} MB read")
