from tianshou_amd.policy.base import BasePolicy
from tianshou_amd.policy.pg import PGPolicy
from tianshou_amd.policy.a2c import A2CPolicy
from tianshou_amd.policy.ppo import PPOPolicy

__all__ = ["BasePolicy", "PGPolicy", "A2CPolicy", "PPOPolicy"]
