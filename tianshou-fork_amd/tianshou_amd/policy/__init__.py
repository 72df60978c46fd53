from tianshou_amd.policy.base import BasePolicy
from tianshou_amd.policy.pg import PGPolicy
from tianshou_amd.policy.a2c import A2CPolicy
from tianshou_amd.policy.ppo import PPOPolicy
from tianshou_amd.policy.npg import NPGPolicy
from tianshou_amd.policy.trpo import TRPOPolicy

__all__ = ["BasePolicy", "PGPolicy", "A2CPolicy", "PPOPolicy", "NPGPolicy", "TRPOPolicy"]
