"""Data-parallel host logic on CPU with world_size-2 and -4 gloo groups (no GPU): gradient
all-reduce (sum and average), all_gather_cat order, and the scaling convention the fused PPO
loss relies on -- per-rank sums divided by the GLOBAL minibatch size, then summed across
ranks -- reproduces the single-process full-batch gradient; the bench's N > 1 self-report
pieces (CollectiveLog call counts and payloads, the replica hash's MAX == MIN check)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import sys
    from tests.conftest import PKG, ROOT
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from tianshou_amd.dist import LOG, DataParallel, param_hash
    LOG.reset()
    dp = DataParallel()
    assert dp.active and dp.world == world and dp.rank == rank
    # all_gather_cat keeps rank order
    g = dp.all_gather_cat(torch.tensor([float(rank), rank + 0.5]))
    assert g.tolist() == [v for r in range(world) for v in (float(r), r + 0.5)]
    # gradient all-reduce: global-mean convention
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(7, 16), torch.nn.Tanh(), torch.nn.Linear(16, 3))
    x = torch.randn(64, 7, generator=torch.Generator().manual_seed(1))
    y = torch.randn(64, 3, generator=torch.Generator().manual_seed(2))
    xs, ys = x[rank::world], y[rank::world]
    b_global = y.numel()  # elements of the global minibatch the mean runs over
    loss = ((net(xs) - ys) ** 2).sum() / b_global  # per-rank sum / global count
    loss.backward()
    dp.all_reduce_grads_(net.parameters())
    grads_sum = [p.grad.clone() for p in net.parameters()]
    for p in net.parameters():
        p.grad = None
    ((net(xs) - ys) ** 2).mean().backward()          # per-rank mean -> average
    dp.all_reduce_grads_(net.parameters(), average=True)
    grads_avg = [p.grad.clone() for p in net.parameters()]
    # advantage moments: (sum, sumsq) all-reduced == full-batch moments
    a = torch.randn(64, dtype=torch.float64, generator=torch.Generator().manual_seed(3))
    mine = a[rank::world]
    sums = dp.all_reduce_(torch.stack([mine.sum(), (mine * mine).sum()]))
    # replicas built from different seeds become rank 0's (A2CPolicy._sync_replicas)
    torch.manual_seed(100 + rank)
    rep = torch.nn.Sequential(torch.nn.Linear(7, 16), torch.nn.Tanh(), torch.nn.Linear(16, 3))
    dp.broadcast_params_(rep.parameters())
    flat = torch.cat([q.detach().reshape(-1) for q in rep.parameters()])
    # replica-consistency hash (bench.py's MAX == MIN check): equal replicas, equal hashes;
    # one flipped bit moves it
    h = param_hash(rep.parameters())
    hmax, hmin = h.clone(), h.clone()
    dist.all_reduce(hmax, op=dist.ReduceOp.MAX)
    dist.all_reduce(hmin, op=dist.ReduceOp.MIN)
    moved = True
    for bit in (0, 31):  # the lowest mantissa bit and the sign bit
        bent = [q.detach().clone() for q in rep.parameters()]
        bent[1].view(-1).view(torch.int32)[3] ^= (1 << bit) if bit < 31 else -(1 << 31)
        moved = moved and int(param_hash(bent)) != int(h)
    # the collective log: logical calls by kind and the last payload of each kind
    log = (dict(LOG.calls), dict(LOG.payload))
    LOG.replayed({"obs_rms": 3})
    LOG.replayed(None)
    replayed = LOG.calls["obs_rms"]
    # ragged all_gather_cat (unequal env shards' ret_rms partials): rank r sends r + 1 values
    rg = dp.all_gather_cat(torch.arange(rank + 1, dtype=torch.float64) + 10 * rank,
                           kind="ret_rms", ragged=True)
    assert rg.tolist() == [10.0 * r + i for r in range(world) for i in range(r + 1)], rg
    # known lengths (the shard table's ret_rms partial counts): no length exchange
    kg = dp.all_gather_known(torch.arange(rank + 1, dtype=torch.float64) + 10 * rank,
                             [r + 1 for r in range(world)], kind="ret_rms")
    assert kg.tolist() == rg.tolist(), kg
    # the once-per-update shard table and the equal-shard requirement of the local-split
    # learn paths (unequal shards must raise, not hang)
    import types
    from tianshou_amd.policy.a2c import A2CPolicy
    stub = types.SimpleNamespace(dp=dp)
    for name in ("_shard_table", "_learn_shards", "_require_equal_shards"):
        setattr(stub, name, types.MethodType(getattr(A2CPolicy, name), stub))
    np.random.seed(7)
    tab = stub._shard_table(100 + rank, 5, torch.device("cpu"))
    assert tab["n"] == [100 + r for r in range(world)] and tab["row_len"] == [5] * world
    assert tab["hash_equal"] and tab["fresh"]
    raised = False
    try:
        stub._require_equal_shards(100 + rank, torch.device("cpu"), "learn")
    except ValueError as e:
        raised = "unequal data-parallel shards" in str(e)
    assert raised and not stub._shards["fresh"]
    stub._require_equal_shards(64, torch.device("cpu"), "learn")  # equal: no error
    np.random.seed(rank)  # different global streams are detected
    assert not stub._shard_table(64, 0, torch.device("cpu"))["hash_equal"]
    out[rank] = (grads_sum, grads_avg, sums, flat, (int(hmax), int(hmin), moved, log, replayed))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_data_parallel_gloo_ranks(world):
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(7, 16), torch.nn.Tanh(), torch.nn.Linear(16, 3))
    x = torch.randn(64, 7, generator=torch.Generator().manual_seed(1))
    y = torch.randn(64, 3, generator=torch.Generator().manual_seed(2))
    ((net(x) - y) ** 2).mean().backward()
    full = [p.grad for p in net.parameters()]
    torch.manual_seed(100)
    rep0 = torch.nn.Sequential(torch.nn.Linear(7, 16), torch.nn.Tanh(), torch.nn.Linear(16, 3))
    want = torch.cat([q.detach().reshape(-1) for q in rep0.parameters()])
    n_grad = sum(q.numel() for q in net.parameters())
    for r in range(world):
        gs, ga, sums, flat, (hmax, hmin, moved, (calls, payload), replayed) = out[r]
        assert torch.equal(flat, want)
        assert hmax == hmin and moved
        assert calls == {"other": 2, "grad": 2, "param_broadcast": 1}
        assert payload["grad"] == ("all_reduce", n_grad, "float32", 4 * n_grad)
        assert payload["param_broadcast"] == ("broadcast", n_grad, "float32", 4 * n_grad)
        assert payload["other"] == ("all_reduce", 2, "float64", 16)
        assert replayed == 3
        for a, b in zip(gs, full):
            np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=1e-5, atol=1e-7)
        for a, b in zip(ga, full):  # equal shards: mean of means == global mean
            np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=1e-5, atol=1e-7)
        a = torch.randn(64, dtype=torch.float64, generator=torch.Generator().manual_seed(3))
        np.testing.assert_allclose(sums.numpy(), [a.sum().item(), (a * a).sum().item()],
                                   rtol=1e-12)
