from tianshou_amd.env.cartpole import CartPoleEnv, CartPoleVectorEnv
from tianshou_amd.env.spaces import Box, Discrete
from tianshou_amd.env.synthetic import DeviceVectorEnv, SyntheticVectorEnv
from tianshou_amd.env.venvs import DummyVectorEnv
from tianshou_amd.env.wrappers import VectorEnvNormObs

__all__ = ["Box", "CartPoleEnv", "CartPoleVectorEnv", "Discrete", "DeviceVectorEnv",
           "DummyVectorEnv", "SyntheticVectorEnv", "VectorEnvNormObs"]
