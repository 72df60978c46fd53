"""Rehearsal of the data-parallel bench path on a one-GPU box: bench.py under
torch.distributed.run with ONE rank, the nccl (= RCCL) backend and --force-dp, so that every
collective of the N>1 path (advantage moments, loss sums, the flat-gradient all-reduce,
the ret_rms all-gather, the max-over-ranks timing) runs through a real RCCL communicator,
next to the HIP-graph replay of the collector steps (captured while the process group and
its watchdog are alive).  The 8-GPU run itself belongs to the driver.

File name sorts first among the GPU tests: this pytest process must not have initialised
HIP when it starts the rank process."""
import json
import os
import socket
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_force_dp_one_rank_rccl():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
           "1", "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "2", "--warmup", "1",
           "--envs", "512", "--T", "128", "--no-cpu-baseline", "--force-dp"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert lines, p.stdout[-2000:]
    out = json.loads(lines[-1])
    assert out["value"] > 0 and out["n_gpus"] == 1
    assert out["config"]["global_batch"] == 512 * 128
    # the RCCL all-reduces were captured into the learn graphs (2048-row minibatches replay
    # whole epochs) and into the collect graphs (global obs_rms), not run eagerly
    assert out["config"]["learn_graph_capture_failed"] is False
    assert "capture failed" not in p.stderr
    # the N > 1 self-report (bench.py data_parallel): collective counts per iteration by
    # kind -- graph-replayed collectives counted per replay --, each kind timed at its
    # payload, per-rank collect / update split, replica consistency
    dpr = out["config"]["data_parallel"]
    assert dpr["rccl_world_size"] == 1
    calls = dpr["collectives_per_iter"]
    T, mb, repeat = 128, 32, 4
    assert calls["obs_rms"] == T  # one per env step (fused step: the int64 totals slot)
    assert calls["grad"] == mb * repeat  # one bucket per minibatch
    assert calls["adv_moments"] == repeat  # one per epoch
    assert calls["ret_rms"] == 1  # one per update
    tim = dpr["collective_timing"]
    for kind in ("obs_rms", "grad", "adv_moments"):
        assert tim[kind]["eager_us"] > 0, kind
        assert tim[kind]["bytes"] > 0, kind
    assert tim["obs_rms"]["dtype"] == "int64"
    assert len(dpr["per_rank_s"]) == 1 and dpr["per_rank_s"][0]["update_s"] > 0
    assert dpr["replica_hash_equal"] is True
