"""Learning-rate schedules of the reference's trainer setup (tianshou/utils/lr_scheduler.py:
MultipleLRSchedulers :8-43, get_linear_lr_schedular :47-56).  BasePolicy.update steps the
scheduler after every learn() (base.py:312-313); the fused Adam reads the learning rate from
a device word refreshed per epoch (FusedActorCritic.set_lr), so captured learn graphs follow
the schedule without being re-captured."""
from typing import Dict, List

import numpy as np
import torch
from torch.optim.lr_scheduler import LambdaLR


class MultipleLRSchedulers:
    """Steps several schedulers together."""

    def __init__(self, *args: torch.optim.lr_scheduler.LambdaLR):
        self.schedulers = args

    def step(self) -> None:
        for scheduler in self.schedulers:
            scheduler.step()

    def state_dict(self) -> List[Dict]:
        return [s.state_dict() for s in self.schedulers]

    def load_state_dict(self, state_dict: List[Dict]) -> None:
        for s, sd in zip(self.schedulers, state_dict):
            s.__dict__.update(sd)


def get_linear_lr_schedular(optim: torch.optim.Optimizer, step_per_epoch: int,
                            step_per_collect: int, epochs: int) -> LambdaLR:
    """Linear decay to 0 over ceil(step_per_epoch / step_per_collect) * epochs updates."""
    max_update_num = np.ceil(step_per_epoch / step_per_collect) * epochs
    return LambdaLR(optim, lr_lambda=lambda epoch: 1 - epoch / max_update_num)
