"""CPU checks of config 1's host side: DummyVectorEnv (venvs.py:260-403) + the CartPole-v1
restatement replay the reference's recorded random-action collect (tests/golden/cartpole.npz)
step for step, the oracle of the device env (oracle/cartpole.py) runs the same dynamics as
the host env, and Batch stacks per-env info dicts like the reference's Batch."""
import os

import numpy as np


def test_dummy_vector_env_replays_reference_collect(golden_dir):
    from tianshou_amd.env import CartPoleEnv, DummyVectorEnv
    z = np.load(os.path.join(golden_dir, "cartpole.npz"))
    E = int(z["E"])
    envs = DummyVectorEnv([CartPoleEnv for _ in range(E)])
    envs.seed(int(z["seed"]))
    obs, infos = envs.reset()
    assert infos == [{}] * E
    np.testing.assert_array_equal(obs, z["c0_data_obs"])
    # the collected rows of env b sit at rows [b*S, b*S + len_b) of the VectorReplayBuffer
    S = len(z["c1_buf_obs"]) // E
    lens = z["c1_lengths"]
    T = int(lens.max())
    cur = obs.copy()
    for t in range(T):
        ids = [b for b in range(E) if t < lens[b]]
        rows = [b * S + t for b in ids]
        np.testing.assert_array_equal(cur[ids], z["c1_buf_obs"][rows])
        o, r, te, tr, info = envs.step(z["c1_buf_act"][rows], ids)
        assert [i["env_id"] for i in info] == ids
        np.testing.assert_array_equal(o, z["c1_buf_obs_next"][rows])
        np.testing.assert_array_equal(r, z["c1_buf_rew"][rows])
        np.testing.assert_array_equal(te, z["c1_buf_terminated"][rows])
        np.testing.assert_array_equal(tr, z["c1_buf_truncated"][rows])
        cur[ids] = o
        done = [b for b, d in zip(ids, te | tr) if d]
        if done:
            ro, _ = envs.reset(done)
            cur[done] = ro


def test_device_env_oracle_runs_host_dynamics():
    from oracle.cartpole import CartPoleHashVecNP
    from tianshou_amd.env import CartPoleEnv
    ora = CartPoleHashVecNP(8, seed=3, max_steps=500)
    ora.reset()
    host = [CartPoleEnv() for _ in range(8)]
    for e, h in enumerate(host):
        h.reset(seed=0)
        h.state = ora.state[e].copy()
    rng = np.random.default_rng(1)
    for _ in range(30):
        a = rng.integers(0, 2, 8)
        wo, wr, wte, wtr = ora.step(a)
        for e, h in enumerate(host):
            if wte[e] and h.steps_beyond_terminated is not None:
                continue
            o, r, te, tr, _ = h.step(a[e])
            np.testing.assert_array_equal(o, wo[e])
            assert (r, te, tr) == (wr[e], wte[e], wtr[e])


def test_batch_stacks_info_dicts():
    from tianshou_amd.data import Batch
    info = np.array([{"env_id": 0, "x": 1.5}, {"env_id": 3, "x": 2.5}], dtype=object)
    b = Batch(info=info)
    assert b.info.env_id.tolist() == [0, 3] and b.info.x.tolist() == [1.5, 2.5]
    b2 = Batch(info=[{}, {}])
    assert b2.info.is_empty()
