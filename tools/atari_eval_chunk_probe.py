"""Per-row time of the no-grad Nature-DQN trunk + heads (process_fn evaluation) at several
chunk sizes (GPU diagnostic).  python tools/atari_eval_chunk_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tianshou-fork_amd")]

from tianshou_amd.utils.net import DiscreteActor, DiscreteCritic  # noqa: E402
from tianshou_amd.utils.net_atari import DQN, layer_init  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = DQN(4, 84, 84, (6,), device=dev, features_only=True, output_dim=512,
              layer_init=layer_init).to(dev)
    actor = DiscreteActor(net, 6, softmax_output=False, device=dev).to(dev)
    critic = DiscreteCritic(net, device=dev).to(dev)
    total = 65536
    obs = torch.randint(0, 256, (total, 4, 84, 84), dtype=torch.uint8, device=dev)
    for c in (2048, 4096, 8192, 16384, 32768, 38043, 65536):
        def run():
            with torch.no_grad():
                for s in range(0, total, c):
                    h, _ = net(obs[s:s + c])
                    actor.last(h)
                    critic.last(h)
        for _ in range(2):
            run()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(3):
            run()
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 3
        print(f"chunk {c:6d}: {ms:8.2f} ms per {total} rows = {ms * 1e3 / total:.3f} us/row",
              flush=True)


if __name__ == "__main__":
    main()
