from tianshou_amd.data.batch import Batch, split_indices, to_numpy, to_torch, to_torch_as
from tianshou_amd.data.buffer import ReplayBuffer, RingIndex, VectorReplayBuffer
from tianshou_amd.data.segtree import SegmentTree
from tianshou_amd.data.prio import PrioritizedReplayBuffer, PrioritizedVectorReplayBuffer
from tianshou_amd.data.collector import Collector

__all__ = ["Batch", "ReplayBuffer", "VectorReplayBuffer", "PrioritizedReplayBuffer",
           "PrioritizedVectorReplayBuffer", "SegmentTree", "RingIndex", "Collector",
           "split_indices", "to_numpy", "to_torch", "to_torch_as"]
