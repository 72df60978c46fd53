"""Round-6 probe (diagnostic): config-1 learn-graph captures per update, device vs host CartPole
envs (python tools/cart_probe.py device|host)."""
import sys, time, torch
sys.path[:0] = [".", "tianshou-fork_amd"]
import bench
from tianshou_amd.policy import ppo as P
caps = []
ncap = [0]
orig = P.PPOPolicy._cat_epoch_graph
orig_cb = P.LOG.capture_begin
def cb(*a, **k):
    ncap[0] += 1
    return orig_cb(*a, **k)
P.LOG.capture_begin = cb
def wrapped(self, fa, obs, arrays, perm, chunks, first):
    c0 = ncap[0]
    r = orig(self, fa, obs, arrays, perm, chunks, first)
    caps.append((obs.data_ptr(), ncap[0] == c0, len(chunks)))
    return r
P.PPOPolicy._cat_epoch_graph = wrapped
sys.argv = ["bench.py", "--workload", "cartpole", "--cartpole-env", sys.argv[1]]
args = bench.parse()
dev = torch.device("cuda", 0)
coll, policy, buf = bench.build_cartpole(args, dev, 0)
for it in range(4):
    torch.cuda.synchronize(); t0 = time.time()
    coll.collect(n_step=args.envs * args.T)
    torch.cuda.synchronize(); t1 = time.time()
    policy.update(0, buf, batch_size=64, repeat=10)
    torch.cuda.synchronize(); t2 = time.time()
    buf.reset()
    n = len(caps); hits = sum(1 for c in caps if c[1])
    print(f"iter {it}: collect {1e3*(t1-t0):.1f} ms update {1e3*(t2-t1):.1f} ms graph calls {n} reused {hits} last obs ptr {caps[-1][0] if caps else None} chunks {caps[-1][2] if caps else None}", flush=True)
    caps.clear()
