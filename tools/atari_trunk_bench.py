"""Timing of the config-5 Nature-DQN trunk on MI355X (diagnostic, not a test):
one 8192-row PPO minibatch forward+backward as two trunk passes (actor and critic, the
reference's formulation) vs one shared pass, and a no-grad evaluation chunk, under
MIOpen's default algorithm choice vs benchmark (find) mode and NCHW vs channels_last.

python tools/atari_trunk_bench.py [--rows 8192] [--iters 10]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tianshou-fork_amd")]

from tianshou_amd.utils.net import DiscreteActor, DiscreteCritic  # noqa: E402
from tianshou_amd.utils.net_atari import DQN, layer_init  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8192)
    ap.add_argument("--eval-rows", type=int, default=32768)  # A2CPolicy._chunks for 4x84x84
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", action="store_true",
                    help="only MIOpen's default choice with channels_last (profiling runs)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for bench_mode in ((False,) if a.only else (False, True)):
        torch.backends.cudnn.benchmark = bench_mode
        for cl in ((True,) if a.only else (False, True)):
            torch.manual_seed(0)
            net = DQN(4, 84, 84, (6,), device=dev, features_only=True, output_dim=512,
                      layer_init=layer_init, channels_last=cl).to(dev)
            actor = DiscreteActor(net, 6, softmax_output=False, device=dev).to(dev)
            critic = DiscreteCritic(net, device=dev).to(dev)
            obs = torch.randint(0, 256, (a.rows, 4, 84, 84), dtype=torch.uint8, device=dev)
            eobs = torch.randint(0, 256, (a.eval_rows, 4, 84, 84), dtype=torch.uint8,
                                 device=dev)
            params = list(actor.parameters()) + list(critic.last.parameters())

            def two_pass():
                x, _ = actor(obs)
                v = critic(obs).flatten()
                (x.sum() + v.sum()).backward()
                for p in params:
                    p.grad = None

            def shared():
                h, _ = net(obs)
                x = actor.last(h)
                v = critic.last(h).flatten()
                (x.sum() + v.sum()).backward()
                for p in params:
                    p.grad = None

            def evaluate():
                with torch.no_grad():
                    h, _ = net(eobs)
                    actor.last(h)
                    critic.last(h)

            t2 = timed(two_pass, a.iters)
            t1 = timed(shared, a.iters)
            te = timed(evaluate, max(2, a.iters // 3))
            print(f"benchmark={bench_mode} channels_last={cl}: minibatch {a.rows} fwd+bwd "
                  f"two-pass {t2:.2f} ms, shared {t1:.2f} ms; eval {a.eval_rows} rows "
                  f"{te:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
