"""Regression test of the HIP-graph-capture abort found in round 4 (commit
a3717f2, tianshou_amd/utils/capture.py): a cyclic-GC pass that runs while a stream is
capturing can free an unreachable ``torch.cuda.CUDAGraph`` whose destructor calls a HIP API
the capture forbids (hipErrorStreamCaptureUnsupported), and the process aborts.

A fresh child process (it has not touched the GPU when it starts) builds a Collector whose
fused collect steps are captured into HIP graphs, drops the collector, and turns its graphs
into cyclic garbage the moment the second collector's capture has begun (a hook on
``CUDAGraph.capture_begin``), with the GC threshold at 1 so that a collection is due at
almost every allocation during the capture.  Inside ``graph_capture`` the cyclic collector
is off, so the graphs are freed after the capture; without it the child aborts.  The
child must exit 0.  Run once per suite: it is not meant to be
repeated to reproduce the fault."""
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

CHILD = r"""
import gc, sys
sys.path.insert(0, sys.argv[1])
import torch
from tianshou_amd.data import Collector, VectorReplayBuffer
from tianshou_amd.env import SyntheticVectorEnv, VectorEnvNormObs
from tianshou_amd.policy import PPOPolicy
from tianshou_amd.utils.models import fixed_std_normal, get_actor_critic, init_and_get_optim

dev = torch.device("cuda", 0)
E, D, A, T = 64, 17, 6, 16


def make():
    env = VectorEnvNormObs(SyntheticVectorEnv(E, (D,), A, ep_len=9, device=dev))
    actor, critic = get_actor_critic((D,), (64, 64), (A,), dev)
    pol = PPOPolicy(actor, critic, init_and_get_optim(actor, critic, 3e-4), fixed_std_normal,
                    action_space=env.action_space).to(dev)
    c = Collector(pol, env, VectorReplayBuffer(E * T, E, device=dev))
    c.graph_steps = 4
    c.collect(n_step=E * T)  # captures the fused-step graphs
    return c


a = make()
pending = [a._graphs]  # the first collector's captured CUDAGraphs, held only from here
assert pending[0], "the first collector captured no HIP graph"
del a
orig_begin = torch.cuda.CUDAGraph.capture_begin


def begin(self, *args, **kwargs):
    # once the stream is capturing, the old graphs become cyclic garbage: only a GC pass can
    # free them, and with threshold 1 one is due at almost every allocation of the capture
    r = orig_begin(self, *args, **kwargs)
    if pending:
        h = [pending.pop()]
        h.append(h)
        del h
    return r


torch.cuda.CUDAGraph.capture_begin = begin
gc.set_threshold(1, 1, 1)
b = make()  # its captures run inside graph_capture
b.collect(n_step=E * T)
torch.cuda.synchronize()
gc.collect()
print("capture-gc ok")
"""


def test_capture_survives_gc_of_unreachable_graphs():
    p = subprocess.run([sys.executable, "-c", CHILD, os.path.join(ROOT, "tianshou-fork_amd")],
                       capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert p.returncode == 0, (p.returncode, p.stderr[-4000:])
    assert "capture-gc ok" in p.stdout
