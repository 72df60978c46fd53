"""Headline benchmark: env-steps/s through Collector.collect + GAE + PPOPolicy.learn
(BASELINE.json metric), config "Synthetic Box(obs=376, act=17), 4096 envs x 2048 steps".

A "step" is one on-policy iteration of the reference trainer (trainer/base.py:552-563):
    collect(n_step=envs*T) -> policy.update(0, buffer, batch_size=envs*T/32, repeat=4)
    -> reset_buffer(keep_statistics=True)
with SURVEY.md §8d's pinned hyper-parameters (Tanh 64-64 actor/critic, Adam 3e-4, gamma .99,
lambda .95, eps_clip .2, vf_coef .25, ent_coef 0, max_grad_norm .5, rew_norm on,
norm_adv on, VectorEnvNormObs on, 32 minibatches, repeat 4).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Multi-GPU = env sharding (weak scaling: every rank runs envs x T of its own), RCCL
all-reduce of gradients / advantage moments / ret_rms partials.  Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "tianshou-fork_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

GAE_BYTES_PER_TRANSITION = 26  # rew f64 8 + v_s 4 + v_s_ 4 + term 1 + trunc 1 + adv 4 + ret 4
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", choices=["humanoid", "small", "atari", "cartpole"],
                    default="humanoid",
                    help="humanoid: BASELINE config 3 (the headline line); small: config 2 "
                         "(Box 17/6, 512 envs x 128 steps); atari: config 5 (u8 4x84x84 frame "
                         "stacks, Discrete(6), Nature-DQN trunk, 1024 envs x 256 steps); "
                         "cartpole: config 1 (CartPole-v1, 4 envs x 500 steps = "
                         "step_per_collect 2000, Net 64-64 shared by Categorical(probs) actor "
                         "and critic, batch 64, repeat 10: test/discrete/test_ppo.py)")
    ap.add_argument("--cartpole-env", choices=["host", "device"], default="host",
                    help="config 1 envs: host = DummyVectorEnv of CartPoleEnv (the reference's "
                         "setup, the Collector's generic host-env loop); device = "
                         "CartPoleVectorEnv (HIP kernel, fused device collect)")
    ap.add_argument("--batch-size", type=int, default=None,
                    help="minibatch rows (default: envs x T / minibatches)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2,
                    help="untimed iterations; the second one completes the collect-graph "
                         "captures (remainder graphs of a new ring phase)")
    ap.add_argument("--envs", type=int, default=None)
    ap.add_argument("--T", type=int, default=None)
    ap.add_argument("--obs", type=int, default=None)
    ap.add_argument("--act", type=int, default=None)
    ap.add_argument("--repeat", type=int, default=4)
    ap.add_argument("--minibatches", type=int, default=32)
    ap.add_argument("--ep-len", type=int, default=None)
    ap.add_argument("--perm", choices=["numpy", "numpy-sorted", "device", "sorted"],
                    default="numpy",
                    help="minibatch permutation: numpy (the reference np.random.permutation "
                         "stream, bit-exact: host MT19937 draws + device shuffle), "
                         "numpy-sorted (the same minibatch sets, rows of each visited in "
                         "ascending buffer order), device (torch.randperm), sorted "
                         "(torch.randperm, rows of each minibatch in ascending order)")
    ap.add_argument("--dp-perm", choices=["global", "local"], default="global",
                    help="data parallel: global = the reference split of the global batch "
                         "(one np.random.permutation(world x n) on every rank), local = "
                         "each rank splits its own rows")
    ap.add_argument("--cpu-steps", type=int, default=None,
                    help="T' of the bounded CPU-baseline sample (envs x T')")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--act-coef", type=float, default=0.0,
                    help="diagnostic: the action-coupled synthetic env (obs = box + c * action, "
                         "not 2^-23-quantised): the fused collect step's general path (env "
                         "after the actor, f64 obs_rms moments); measures what the synthetic "
                         "env's two shortcuts buy")
    ap.add_argument("--obs-pad", choices=["on", "off"], default="on",
                    help="diagnostic: off stores the 376-float observation rows unpadded "
                         "(VectorReplayBuffer.PAD_MIN; default: 128-byte row pitch)")
    ap.add_argument("--exact-obs-rms", action="store_true",
                    help="VectorEnvNormObs with the reference's f32 obs_rms arithmetic bit for "
                         "bit (sequential f32 column sums; opt-in, measures its cost)")
    ap.add_argument("--exact-pipeline", type=int, default=None,
                    help="with --exact-obs-rms: env rows computed this many steps ahead and the "
                         "f32 statistic on a second graph branch (Collector.exact_pipeline, "
                         "default 5; 0: serial, one exact update between step launches)")
    ap.add_argument("--exact-group", type=int, default=None,
                    help="diagnostic: steps per statistics launch of the pipelined exact "
                         "obs_rms (Collector.exact_group, default 2)")
    ap.add_argument("--exact-branches", type=int, default=None,
                    help="diagnostic: concurrent statistics streams of the pipelined exact "
                         "obs_rms (Collector.exact_branches; one when groups > 1)")
    ap.add_argument("--force-dp", action="store_true",
                    help="diagnostic: under torch.distributed.run with ONE rank, run the "
                         "data-parallel code path (RCCL collectives over a one-rank "
                         "communicator) -- rehearses the N>1 path on a one-GPU box")
    ap.add_argument("--graph-learn", choices=["auto", "on", "off"], default="auto",
                    help="learn() epochs from captured HIP graphs: auto = only for minibatches "
                         "< 65536 rows (PPOPolicy default); on at the headline shape measured "
                         "~5 %% slower per update than eager launches")
    a = ap.parse_args()
    defaults = dict(humanoid=(4096, 2048, 376, 17, 256, 1000),
                    small=(512, 128, 17, 6, 128, 1000),
                    atari=(1024, 256, 0, 6, 16, 256),
                    cartpole=(4, 500, 4, 2, 0, 500))[a.workload]
    for k, v in zip(("envs", "T", "obs", "act", "cpu_steps", "ep_len"), defaults):
        if getattr(a, k) is None:
            setattr(a, k, v)
    if a.workload in ("atari", "cartpole"):
        a.no_cpu_baseline = True  # the CPU port covers the Box workloads only
    if a.workload == "cartpole":
        if a.batch_size is None:
            a.batch_size = 64
        if "--repeat" not in " ".join(sys.argv):
            a.repeat = 10
    return a


class GaeTimer:
    """HIP-event timing of every tsrl_gae launch, on the stream it is launched on: the two
    events are handed to the library (tsrl_gae_time_next), which launches the GAE kernel with
    hipExtLaunchKernel so that the events record the kernel's OWN start and stop -- the
    duration rocprof reports, without the dispatch latency an event pair recorded around the
    launch also holds (round 4-5: 44-58 us by such a pair vs 38-44 us by rocprof)."""

    def __init__(self):
        self.events = []
        self.n = 0
        self.on = False

    def __call__(self, phase, n):
        if not self.on or phase != "start":
            return
        from tianshou_amd import _C
        pair = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
        for ev in pair:  # create the events (torch creates them at their first record)
            ev.record(torch.cuda.current_stream())
        _C.check(_C.lib().tsrl_gae_time_next(pair[0].cuda_event, pair[1].cuda_event),
                 "tsrl_gae_time_next")
        self.events.append(pair)
        self.n = n

    def each_ms(self):
        return [a.elapsed_time(b) for a, b in self.events if b is not None]

    def mean_ms(self):
        ts = self.each_ms()
        return float(np.mean(ts)) if ts else float("nan")


def gae_pmc_traffic(E: int, T: int):
    """(HBM bytes per GAE launch, note) from the committed rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes of the same kernel and shape (FETCH doubled per the gfx950
    calibration).  PMC collection needs the profiler, so the bench does not re-measure it;
    the record names the sha256 of the kernel source it was measured on, and a different
    csrc/gae.hip makes the figure stale: then traffic is null and the note says why."""
    import hashlib
    import glob
    if (E, T) != (4096, 2048):
        return None, "no PMC record for this shape"
    src = os.path.join(ROOT, "tianshou-fork_amd", "csrc", "gae.hip")
    with open(src, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()
    for pmc in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_gae_pmc.json")), reverse=True):
        with open(pmc) as f:
            d = json.load(f)["derived"]
        if d.get("source_sha256") == sha:
            return d["traffic_bytes"], f"{os.path.relpath(pmc, ROOT)} (gae.hip sha256 {sha[:12]})"
    return None, (f"stale: no profiles/r*_gae_pmc.json measured on this gae.hip "
                  f"(sha256 {sha[:12]}); re-run tools/pmc_gae.py")


def build_atari(args, dev, rank):
    """BASELINE config 5: examples/atari/atari_ppo.py's PPO (shared Nature-DQN trunk,
    Categorical(logits), frame-stack buffer with save_only_last_obs / ignore_obs_next) on the
    device u8 env with FrameStack semantics; no obs normalisation (the net scales by 1/255)."""
    from tianshou_amd.data import Collector, VectorReplayBuffer
    from tianshou_amd.env import Discrete, SyntheticVectorEnv
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.net import ActorCritic, DiscreteActor, DiscreteCritic
    from tianshou_amd.utils.net_atari import DQN, layer_init
    E, T, A = args.envs, args.T, args.act
    env = SyntheticVectorEnv(E, (4, 84, 84), A, ep_len=args.ep_len, seed=rank, device=dev,
                             obs_dtype=np.uint8, discrete=True, frame_stack=4)
    net = DQN(4, 84, 84, (A,), device=dev, features_only=True, output_dim=512,
              layer_init=layer_init).to(dev)
    actor = DiscreteActor(net, A, softmax_output=False, device=dev).to(dev)
    critic = DiscreteCritic(net, device=dev).to(dev)
    optim = torch.optim.Adam(ActorCritic(actor, critic).parameters(), lr=2.5e-4, eps=1e-5)
    policy = PPOPolicy(actor, critic, optim,
                       lambda p: torch.distributions.Categorical(logits=p),
                       action_space=Discrete(A), action_scaling=False, discount_factor=0.99,
                       gae_lambda=0.95, max_grad_norm=0.5, vf_coef=0.25, ent_coef=0.01,
                       eps_clip=0.1, value_clip=True, dual_clip=None,
                       advantage_normalization=False, recompute_advantage=False,
                       reward_normalization=False,
                       perm_device=args.perm in ("device", "sorted")).to(dev)
    buf = VectorReplayBuffer(E * T, E, stack_num=4, ignore_obs_next=True,
                             save_only_last_obs=True, device=dev)
    return Collector(policy, env, buf, exploration_noise=True), policy, buf


def spawn_ranks(n: int) -> int:
    """``--gpus N`` without a launcher: start N rank processes of this script (one per GPU,
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment) before this process
    touches the GPU; rank 0 prints the JSON line.  Returns the worst exit code."""
    import socket
    import subprocess
    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rcs = [p.wait() for p in procs]
    return max(abs(rc) for rc in rcs)


def build_cartpole(args, dev, rank):
    """BASELINE config 1: test/discrete/test_ppo.py's PPO (Net 64-64 shared by the
    Categorical(probs) actor and the critic, orthogonal init, Adam 3e-4, vf .5, ent 0,
    max_grad_norm .5, gae .95, no rew/adv normalisation) over 4 CartPole-v1 envs."""
    from tianshou_amd.data import Collector, VectorReplayBuffer
    from tianshou_amd.env import CartPoleEnv, CartPoleVectorEnv, Discrete, DummyVectorEnv
    from tianshou_amd.policy import PPOPolicy
    from tianshou_amd.utils.net import ActorCritic, DiscreteActor, DiscreteCritic, Net
    E = args.envs
    if args.cartpole_env == "host":
        env = DummyVectorEnv([CartPoleEnv for _ in range(E)])
        env.seed(1626 + 1000 * rank)
    else:
        env = CartPoleVectorEnv(E, seed=1626 + rank, device=dev)
    net = Net(4, hidden_sizes=(64, 64), device=dev)
    actor = DiscreteActor(net, 2, device=dev).to(dev)
    critic = DiscreteCritic(net, device=dev).to(dev)
    ac = ActorCritic(actor, critic)
    for m in ac.modules():
        if isinstance(m, torch.nn.Linear):
            torch.nn.init.orthogonal_(m.weight)
            torch.nn.init.zeros_(m.bias)
    optim = torch.optim.Adam(ac.parameters(), lr=3e-4)
    policy = PPOPolicy(actor, critic, optim, torch.distributions.Categorical,
                       discount_factor=0.99, max_grad_norm=0.5, eps_clip=0.2, vf_coef=0.5,
                       ent_coef=0.0, gae_lambda=0.95, reward_normalization=False,
                       dual_clip=None, value_clip=False, action_space=Discrete(2),
                       deterministic_eval=True, advantage_normalization=False,
                       recompute_advantage=False, action_scaling=False,
                       perm_device=args.perm in ("device", "sorted")).to(dev)
    buf = VectorReplayBuffer(20000, E, device=dev)
    return Collector(policy, env, buf), policy, buf


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    distributed = world > 1 or (args.force_dp and "WORLD_SIZE" in os.environ)
    if distributed:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)
        if dist.get_world_size() != args.gpus:
            print(f"bench.py: RCCL world size {dist.get_world_size()} != --gpus {args.gpus}",
                  file=sys.stderr)
            sys.exit(2)
        if args.force_dp:
            from tianshou_amd.dist import DataParallel
            DataParallel.force = True

    from tianshou_amd.data import Collector, VectorReplayBuffer
    from tianshou_amd.env import SyntheticVectorEnv, VectorEnvNormObs
    from tianshou_amd.policy import PPOPolicy, base as pbase
    if args.obs_pad == "off":
        VectorReplayBuffer.PAD_MIN = 1 << 30
    from tianshou_amd.utils.models import fixed_std_normal, get_actor_critic, init_and_get_optim

    torch.manual_seed(0)  # identical network init on every rank (the policy also
    # broadcasts rank 0's parameters before its first update); one global np.random
    # stream on every rank: the reference permutation of the global batch
    np.random.seed(0 if args.dp_perm == "global" else rank)
    E, T, D, A = args.envs, args.T, args.obs, args.act
    n = E * T
    if args.workload == "atari":
        coll, policy, buf = build_atari(args, dev, rank)
        D = "4x84x84 u8"
    elif args.workload == "cartpole":
        coll, policy, buf = build_cartpole(args, dev, rank)
    else:
        env = VectorEnvNormObs(SyntheticVectorEnv(E, (D,), A, ep_len=args.ep_len, seed=rank,
                                                  device=dev, act_coef=args.act_coef),
                               exact_obs_rms=args.exact_obs_rms)
        actor, critic = get_actor_critic((D,), (64, 64), (A,), dev)
        # to the device before the optimiser: fused + capturable Adam
        actor, critic = actor.to(dev), critic.to(dev)
        optim = init_and_get_optim(actor, critic, 3e-4)
        policy = PPOPolicy(actor, critic, optim, fixed_std_normal,
                           action_space=env.action_space, discount_factor=0.99,
                           gae_lambda=0.95, max_grad_norm=0.5, vf_coef=0.25, ent_coef=0.0,
                           reward_normalization=True, advantage_normalization=True,
                           recompute_advantage=False, eps_clip=0.2, value_clip=False,
                           dual_clip=None, action_bound_method="clip",
                           perm_device=args.perm in ("device", "sorted")).to(dev)
        buf = VectorReplayBuffer(n, E, device=dev)
        coll = Collector(policy, env, buf)
        if args.exact_pipeline is not None:
            coll.exact_pipeline = args.exact_pipeline
        if args.exact_branches is not None:
            coll.exact_branches = args.exact_branches
        if args.exact_group is not None:
            coll.exact_group = args.exact_group
    torch.manual_seed(rank)  # per-rank action sampling streams
    policy.graph_learn = {"auto": None, "on": True, "off": False}[args.graph_learn]
    policy.sort_minibatch = args.perm in ("sorted", "numpy-sorted")
    # global (default): every rank draws the reference np.random.permutation of the
    # world x n global rows and keeps its share (threaded host draws prefetched during the
    # collect, device resolution on a side stream); local: per-rank splits
    policy.dp_permutation = args.dp_perm
    timer = GaeTimer()
    pbase.GAE_HOOK = timer
    phase = {"collect": 0.0, "update": 0.0}

    def iteration():
        t0 = time.perf_counter()
        coll.collect(n_step=n)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        policy.update(0, buf, batch_size=args.batch_size or n // args.minibatches,
                      repeat=args.repeat)
        coll.reset_buffer(keep_statistics=True)
        torch.cuda.synchronize()
        phase["collect"] += t1 - t0
        phase["update"] += time.perf_counter() - t1

    def barrier():
        if distributed:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        iteration()
    phase.update(collect=0.0, update=0.0)
    from tianshou_amd import dist as tdist
    tdist.LOG.reset()  # collectives of the timed iterations only
    timer.on = True
    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        iteration()
        if rank == 0:
            print(f"# iter {i} collect {phase['collect'] / (i + 1):.3f}s "
                  f"update {phase['update'] / (i + 1):.3f}s", file=sys.stderr, flush=True)
    barrier()
    elapsed = time.perf_counter() - t0
    timer.on = False
    if distributed:
        import torch.distributed as dist
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    dp_report = None
    if distributed:
        # N > 1 self-report (rank-collective; every rank takes part): per-iteration counts of
        # each collective kind in the timed region, each kind timed at its payload, the
        # collect / update split of every rank, and replica consistency (parameter hash
        # all-reduced MAX == MIN)
        import torch.distributed as dist
        calls = {k: v / args.steps for k, v in sorted(tdist.LOG.calls.items())}
        split = torch.tensor([phase["collect"] / args.steps, phase["update"] / args.steps],
                             dtype=torch.float64, device=dev)
        per_rank = [torch.empty_like(split) for _ in range(world)]
        dist.all_gather(per_rank, split)
        h = tdist.param_hash(list(policy.parameters()))
        hmax, hmin = h.clone(), h.clone()
        dist.all_reduce(hmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(hmin, op=dist.ReduceOp.MIN)
        probe = tdist.probe_collectives(tdist.default_dp())
        dp_report = {
            "rccl_world_size": dist.get_world_size(),
            "collectives_per_iter": calls,
            "collective_timing": probe,
            "per_rank_s": [{"rank": r, "collect_s": round(float(t[0]), 5),
                            "update_s": round(float(t[1]), 5)} for r, t in enumerate(per_rank)],
            "replica_hash_equal": bool(int(hmax) == int(hmin)),
            "param_hash": int(h),
        }
    total_steps = n * world * args.steps
    value = total_steps / elapsed
    gae_ms = timer.mean_ms()
    gae_bytes = GAE_BYTES_PER_TRANSITION * n
    achieved = gae_bytes / (gae_ms * 1e-3) / 1e9
    traffic, traffic_note = gae_pmc_traffic(E, T)
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            from oracle import cpu_port
            threads = min(16, os.cpu_count() or 1)
            v, dt = cpu_port.run_iteration(E, args.cpu_steps, D, A, repeat=args.repeat,
                                           minibatches=args.minibatches, ep_len=args.ep_len,
                                           threads=threads)
            cpu = {"value": v, "unit": "env-steps/s", "cores": threads, "kind": "port",
                   "sample": f"one iteration of {E} envs x {args.cpu_steps} steps "
                             f"(Box {D}/{A}), build CPU restatement "
                             f"(oracle/cpu_port.py: NumPy env+obs-norm+buffer, C GAE, "
                             f"torch-CPU PPO), {dt:.1f}s; parity-checked against the "
                             f"reference Collector + VectorEnvNormObs + process_fn goldens "
                             f"(tests/test_oracle.py::test_cpu_port_matches_reference_"
                             f"collector)"}
        line = {
            "metric": "env-steps/sec through collect+GAE+PPO.learn",
            "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32 (GAE scan f64)", "data": "synthetic",
            "config": {"workload": (f"CartPole-v1 ({args.cartpole_env} envs)"
                                    if args.workload == "cartpole" else
                                    f"Synthetic {'Discrete' if args.workload == 'atari' else 'Box'}"
                                    f"(obs={D}, act={A})") +
                                   f", {E} envs x {T} steps "
                                   f"per GPU, GAE+PPO (repeat {args.repeat}, "
                                   f"minibatch {args.batch_size or n // args.minibatches})",
                       "baseline_config": dict(humanoid=3, small=2, atari=5,
                                               cartpole=1)[args.workload],
                       "envs_per_gpu": E, "steps_per_env": T, "global_batch": n * world,
                       "minibatch": (args.batch_size or n // args.minibatches) * world,
                       "parallelism": f"env-sharded dp{world}",
                       "permutation": args.perm + (f" ({args.dp_perm} over {world} ranks)"
                                                   if world > 1 or args.force_dp else ""),
                       "rccl_world_size": world if distributed else None,
                       "learn_graph": args.graph_learn,
                       "obs_rms": ("exact f32 (reference arithmetic), " + (
                           f"pipelined {coll.exact_pipeline} steps ahead, statistics "
                           f"{coll._xpipe_group()} steps per launch"
                           if coll._xpipe_ok() else "serial")) if args.exact_obs_rms
                       else ("f64 moments (atomic), action-coupled env" if args.act_coef
                             else "exact int64 moments (quantised synthetic obs), f64 merge"),
                       "learn_graph_capture_failed": bool(getattr(policy, "_graph_failed",
                                                                  False)),
                       "collect_s": phase["collect"] / args.steps,
                       "update_s": phase["update"] / args.steps,
                       "data_parallel": dp_report},
            "roofline": {"kernel": "tsrl_gae (gae_rows_staged_kernel)", "bound": "hbm",
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_note,
                         "launch_us": gae_ms * 1e3,
                         "launch_us_each": [round(t * 1e3, 2) for t in timer.each_ms()],
                         "bytes_per_launch": gae_bytes},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if distributed:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
