from tianshou_amd.env.spaces import Box, Discrete
from tianshou_amd.env.synthetic import DeviceVectorEnv, SyntheticVectorEnv
from tianshou_amd.env.wrappers import VectorEnvNormObs

__all__ = ["Box", "Discrete", "DeviceVectorEnv", "SyntheticVectorEnv", "VectorEnvNormObs"]
