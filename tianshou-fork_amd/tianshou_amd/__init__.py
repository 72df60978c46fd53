"""tianshou_amd -- MI355X-native on-policy hot path of tianshou 0.5.1:
Collector -> device VectorReplayBuffer -> GAE -> PPOPolicy.learn, with the reference's
class API on top of the libtsrl HIP kernels (include/tsrl.h)."""
__version__ = "0.1.0"

from tianshou_amd import data, env, policy, utils  # noqa: F401,E402
