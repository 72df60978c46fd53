"""Worker for tests/test_gpu_a_dist.py::test_unequal_env_shards: data parallelism with
UNEQUAL env shards (rank 0 48 envs, rank 1 80 envs; ADVICE r03: the obs_rms row count rides
the int64 totals slot, so each step's global merge counts every rank's rows) on the fused
collect step at D = 376 over gloo, then one PPO update with the reference's split of the
GLOBAL batch (every rank draws np.random.permutation of the 128 * T global rows and keeps
its own; global minibatches of world * batch_size rows).  Rank 0 receives rank 1's buffer,
builds the union buffer (rank 0's envs first: the env-major order of one
VectorReplayBuffer over all 128 envs) and runs the single-process update over it with the
same initial networks and np.random stream; it saves both results and the global obs_rms.

    python tests/dist_unequal_worker.py RANK WORLD PORT OUTDIR
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tianshou-fork_amd"))

SHARDS, T, D, A, L, BS = (48, 80), 32, 376, 17, 9, 256
KEYS = ("obs", "obs_next", "act", "rew", "terminated", "truncated", "done")
PF = ("v_s", "returns", "adv", "logp_old")


def _capture(policy):
    """Keep a CPU copy of process_fn's outputs (diagnostics of the comparison)."""
    cap, orig = {}, policy.process_fn

    def pf(batch, buffer, indices):
        out = orig(batch, buffer, indices)
        cap.update({k: out[k].detach().reshape(-1).float().cpu() for k in PF})
        return out
    policy.process_fn = pf
    return cap


def main():
    rank, world, port, outdir = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    assert world == len(SHARDS)
    import numpy as np
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = port
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    from dist_c4_worker import build
    import dist_c4_worker
    from tianshou_amd.data import Batch, Collector, VectorReplayBuffer
    from tianshou_amd.dist import DataParallel
    from tianshou_amd.env import SyntheticVectorEnv, VectorEnvNormObs

    dist_c4_worker.D, dist_c4_worker.A = D, A
    E = SHARDS[rank]
    n = E * T
    policy = build(dev)
    env = VectorEnvNormObs(SyntheticVectorEnv(E, (D,), A, ep_len=L, seed=rank, device=dev))
    buf = VectorReplayBuffer(n, E, device=dev)
    coll = Collector(policy, env, buf, sync_obs_rms=True)
    torch.manual_seed(100 + rank)
    coll.collect(n_step=n)
    assert coll._step_on, "the fused one-launch step did not run"
    rms = env.get_obs_rms()
    rms_state = (torch.as_tensor(rms.mean), torch.as_tensor(rms.var), float(rms.count))
    cap = _capture(policy)
    np.random.seed(0)  # one global np.random stream: the reference split of the global batch
    res = policy.update(0, buf, batch_size=BS, repeat=1)
    sd = {k: v.detach().cpu() for k, v in policy.state_dict().items()}
    if rank != 0:
        for k in KEYS:
            t = getattr(buf, k).contiguous()
            # host copies: gloo moves host tensors (a CUDA tensor's copy is not ordered
            # with this process's streams)
            dist.send((t.to(torch.uint8) if t.dtype == torch.bool else t).cpu(), 0)
        dist.send(rms_state[0].cpu(), 0)
        dist.send(rms_state[1].cpu(), 0)
        for k in PF:
            dist.send(cap[k], 0)
        dist.barrier()
        dist.destroy_process_group()
        return
    parts = {k: [getattr(buf, k).contiguous()] for k in KEYS}
    for r in range(1, world):
        for k in KEYS:
            like = getattr(buf, k)
            shape = (SHARDS[r] * T,) + tuple(like.shape[1:])
            t = torch.empty(shape, dtype=torch.uint8 if like.dtype == torch.bool
                            else like.dtype)
            dist.recv(t, r)
            t = t.to(like.device)
            parts[k].append(t.bool() if like.dtype == torch.bool else t)
    other = [torch.empty(D), torch.empty(D)]
    dist.recv(other[0], 1)
    dist.recv(other[1], 1)
    pf = {k: [cap[k]] for k in PF}
    for k in PF:
        t = torch.empty(SHARDS[1] * T, dtype=cap[k].dtype)
        dist.recv(t, 1)
        pf[k].append(t)
    dist.barrier()
    dist.destroy_process_group()
    del coll, env
    NE = sum(SHARDS)
    union = VectorReplayBuffer(NE * T, NE, device=dev)
    union.set_batch(Batch(**{k: torch.cat(v) for k, v in parts.items()}))
    del parts
    ring = union._ring
    ring.lengths[:] = T
    ring.index[:] = 0
    ring.last_index = ring.offset + T - 1
    ref = build(dev)
    ref.dp = DataParallel()
    ref.dp.enabled = False
    cap_ref = _capture(ref)
    np.random.seed(0)
    res_ref = ref.update(0, union, batch_size=world * BS, repeat=1)
    sd_ref = {k: v.detach().cpu() for k, v in ref.state_dict().items()}
    terms = ("loss", "loss/clip", "loss/vf", "loss/ent")
    torch.save(dict(loss=torch.tensor([res[k] for k in terms]),
                    loss_ref=torch.tensor([res_ref[k] for k in terms]),
                    sd=sd, sd_ref=sd_ref, rms_mean=rms_state[0], rms_var=rms_state[1],
                    rms_count=rms_state[2], rms_mean1=other[0], rms_var1=other[1],
                    pf={k: torch.cat(v) for k, v in pf.items()}, pf_ref=cap_ref),
               os.path.join(outdir, "uneq.pt"))


if __name__ == "__main__":
    main()
