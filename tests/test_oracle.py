"""Pin the CPU oracle to the reference's own outputs (tests/golden, made by
tools/gen_goldens.py from /root/reference).  CPU only."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import ref, synth_env


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def test_gae_known_answers(golden_dir):
    """test/base/test_returns.py:22-112 vectors, bit-exact in f64."""
    z = _load(golden_dir, "returns_known.npz")
    for c in range(int(z["ncases"])):
        p = f"c{c}_"
        v = z[p + "v_next"] if bool(z[p + "has_v"]) else None
        ret, adv = ref.compute_episodic_return(
            z[p + "rew"], z[p + "term"], z[p + "trunc"], z[p + "indices"], z[p + "unfinished"],
            v, None, float(z[p + "gamma"]), float(z[p + "lam"]))
        assert np.array_equal(ret, z[p + "returns"]), c
        assert np.array_equal(adv, z[p + "adv"]), c


@pytest.mark.parametrize("tag", ["full", "wrap", "part"])
def test_gae_random_bitexact(golden_dir, tag):
    z = _load(golden_dir, "gae_random.npz")
    p = tag + "_"
    ret, adv = ref.compute_episodic_return(
        z[p + "rew"], z[p + "term"], z[p + "trunc"], z[p + "indices"], z[p + "unfinished"],
        z[p + "v_s_"], z[p + "v_s"], 0.99, 0.95)
    assert np.array_equal(adv, z[p + "adv"])
    assert np.array_equal(ret, z[p + "returns"])
    s = np.float64(z[p + "scale"])
    ret, adv = ref.compute_episodic_return(
        z[p + "rew"], z[p + "term"], z[p + "trunc"], z[p + "indices"], z[p + "unfinished"],
        z[p + "v_s_"] * s, z[p + "v_s"] * s, 0.99, 0.95)
    assert np.array_equal(adv, z[p + "adv_scaled"])
    assert np.array_equal(ret, z[p + "returns_scaled"])


@pytest.mark.parametrize("name", ["manager", "ragged"])
def test_buffer_index_math(golden_dir, name):
    """test/base/test_buffer.py:701-901 sequence + ragged random trace, bit-exact."""
    with open(os.path.join(golden_dir, "buffer_traces.json")) as f:
        tr = json.load(f)[name]
    buf = ref.VecBufferIndex(tr["total"], tr["num"])
    allidx = np.arange(buf.maxsize)
    for step in tr["trace"]:
        if step["op"] == "add":
            d = step["data"]
            ptr, ep_rew, ep_len, ep_idx = buf.add(np.asarray(d["rew"], float),
                                                  np.asarray(d["terminated"]),
                                                  np.asarray(d["truncated"]), step["ids"])
            assert ptr.tolist() == step["ptr"]
            assert ep_rew.tolist() == step["ep_rew"]
            assert ep_len.tolist() == step["ep_len"]
            assert ep_idx.tolist() == step["ep_idx"]
        else:
            buf.reset(step["keep"])
        st = step["state"]
        assert buf.sample_indices0().tolist() == st["sample0"]
        assert buf.prev(allidx).tolist() == st["prev"]
        assert buf.next(allidx).tolist() == st["next"]
        assert buf.unfinished_index().tolist() == st["unfinished"]
        assert len(buf) == st["len"]
        assert buf.last_index.tolist() == st["last_index"]
        assert buf.sizes.tolist() == st["lengths"]
        if st["done"]:
            assert buf.done.astype(int).tolist() == st["done"]


def test_split_table(golden_dir):
    with open(os.path.join(golden_dir, "split.json")) as f:
        g = json.load(f)
    for c in g["cases"]:
        if c["seed"] is not None:
            np.random.seed(c["seed"])
        parts = ref.split_parts(c["n"], c["size"], c["shuffle"], c["merge_last"])
        assert [p.tolist() for p in parts] == c["parts"], c
    np.random.seed(3)
    big = np.random.permutation(1 << 16)
    assert big[:64].tolist() == g["perm_seed3_n65536_head"]
    assert int((big * np.arange(1 << 16)).sum()) == g["perm_seed3_n65536_wsum"]


def test_rms(golden_dir):
    z = _load(golden_dir, "rms.npz")
    r = ref.RMS()
    for i in range(int(z["n"])):
        r.update(z[f"x{i}"])
        assert np.array_equal(np.asarray(r.mean), z[f"mean{i}"])
        assert np.array_equal(np.asarray(r.var), z[f"var{i}"])
        assert r.count == int(z[f"count{i}"])
        assert np.array_equal(r.norm(z[f"x{i}"]), z[f"norm{i}"])


def test_synth_env_through_reference_collector(golden_dir):
    """The synthetic env restated in NumPy reproduces what the reference Collector stored
    (rew / flags exactly; obs after the reference's own VectorEnvNormObs)."""
    z = _load(golden_dir, "collector.npz")
    E, D, L, T = (int(z[k]) for k in ("E", "D", "L", "T"))
    env = synth_env.SynthVecEnvNP(E, (D,), int(z["A"]), L)
    rms = ref.RMS()
    obs = env.reset()
    rms.update(obs)
    obs = rms.norm(obs)
    store = {k: np.zeros((E, T) + s, dt) for k, s, dt in
             (("obs", (D,), np.float32), ("obs_next", (D,), np.float32),
              ("rew", (), np.float64), ("term", (), bool), ("trunc", (), bool))}
    for t in range(T):
        nxt, rew, term, trunc = env.step()
        rms.update(nxt)
        nxt = rms.norm(nxt)
        store["obs"][:, t], store["obs_next"][:, t] = obs, nxt
        store["rew"][:, t], store["term"][:, t], store["trunc"][:, t] = rew, term, trunc
        done = np.flatnonzero(term | trunc)
        obs = nxt.copy()
        if len(done):
            r = env.reset(done)
            rms.update(r)
            obs[done] = rms.norm(r)
    assert np.array_equal(store["rew"].reshape(-1), z["c1_buf_rew"])
    assert np.array_equal(store["term"].reshape(-1), z["c1_buf_terminated"])
    assert np.array_equal(store["trunc"].reshape(-1), z["c1_buf_truncated"])
    assert np.array_equal(store["obs"].reshape(-1, D), z["c1_buf_obs"])
    assert np.array_equal(store["obs_next"].reshape(-1, D), z["c1_buf_obs_next"])
    assert np.array_equal(np.asarray(rms.mean), z["c1_rms_mean"])
    assert rms.count == int(z["c1_rms_count"])


def test_ppo_loss_oracle_matches_reference_grads(golden_dir):
    """One full-batch PPO minibatch through the torch-fp32 loss restatement reproduces the
    reference's recorded gradients (wrt the actor head/critic head outputs are implied by
    the parameter grads; here we check the loss values via a tiny re-run of the nets)."""
    z = _load(golden_dir, "ppo_learn.npz")
    cfg = json.loads(str(z["base_cfg"]))
    assert cfg["n"] == cfg["batch_size"] and cfg["repeat"] == 1
    from tianshou_amd.utils.net import build_actor_critic_from_state
    actor, critic = build_actor_critic_from_state(
        {k[len("base_init_"):]: torch.as_tensor(z[k]) for k in z.files
         if k.startswith("base_init_")}, device="cpu")
    obs = torch.as_tensor(z["base_obs"])
    (mu, _), _ = actor(obs)
    value = critic(obs).flatten()
    loss, clip, vf, ent, g = ref.ppo_gaussian_loss_torch(
        mu, actor.sigma_param.detach().flatten(), value, torch.as_tensor(z["base_act"]),
        torch.as_tensor(z["base_logp_old"]), torch.as_tensor(z["base_adv"]),
        torch.as_tensor(z["base_returns"]), torch.as_tensor(z["base_v_s"]),
        vf_coef=0.25, ent_coef=0.0)
    np.testing.assert_allclose(float(clip), float(z["base_loss_clip"][0]), rtol=1e-5)
    np.testing.assert_allclose(float(vf), float(z["base_loss_vf"][0]), rtol=1e-5)
    np.testing.assert_allclose(float(ent), float(z["base_loss_ent"][0]), rtol=1e-5)


STACK_CASES = [("atari", 4, True, True, False), ("avail", 4, True, True, True),
               ("full_obs", 3, False, False, False), ("last_next", 3, True, False, True)]


def replay_stack_case(z, name, last_only, ign_next):
    """Re-run the golden add sequence through the oracle's index restatement; returns the
    index object and the stored obs / obs_next arrays (manager.py:104-161)."""
    p = name + "_"
    num, per = 5, 8
    ix = ref.VecBufferIndex(num * per, num)
    frame = z[p + "in_obs"].shape[2:] if last_only else z[p + "in_obs"].shape[1:]
    obs = np.zeros((ix.maxsize,) + frame, np.uint8)
    obs_next = np.zeros_like(obs)
    o = 0
    for step, k in enumerate(z[p + "sizes"]):
        sl = slice(o, o + k)
        o += k
        ids = z[p + "ids"][sl]
        gptr, _, _, _ = ix.add(z[p + "in_rew"][sl], z[p + "in_term"][sl], z[p + "in_trunc"][sl],
                               ids)
        ob, obn = z[p + "in_obs"][sl], z[p + "in_obs_next"][sl]
        obs[gptr] = ob[:, -1] if last_only else ob
        obs_next[gptr] = obn[:, -1] if last_only else obn
        if step == 40:
            ix.reset(keep_statistics=True)
    return ix, obs, (None if ign_next else obs_next)


@pytest.mark.parametrize("name,stack_num,last_only,ign_next,avail", STACK_CASES)
def test_frame_stack_oracle(golden_dir, name, stack_num, last_only, ign_next, avail):
    """oracle.stack_get / avail_indices vs the reference's VectorReplayBuffer with
    stack_num / save_only_last_obs / ignore_obs_next / sample_avail (tools/gen_goldens.py
    gen_stack), bit-exact."""
    z = np.load(os.path.join(golden_dir, "stack.npz"))
    p = name + "_"
    ix, obs, obs_next = replay_stack_case(z, name, last_only, ign_next)
    assert np.array_equal(obs, z[p + "stored_obs"])
    if obs_next is not None:
        assert np.array_equal(obs_next, z[p + "stored_obs_next"])
    allidx = np.arange(ix.maxsize)
    assert np.array_equal(ix.prev(allidx), z[p + "prev"])
    assert np.array_equal(ix.next(allidx), z[p + "next"])
    q = z[p + "q_idx"]
    assert np.array_equal(ref.stack_get(obs, q, stack_num, ix.prev), z[p + "q_obs"])
    want_next = ref.stack_get(obs, ix.next(q), stack_num, ix.prev) if obs_next is None else \
        ref.stack_get(obs_next, q, stack_num, ix.prev)
    assert np.array_equal(want_next, z[p + "q_obs_next"])
    if avail:
        assert np.array_equal(ref.avail_indices(ix, stack_num), z[p + "sample0"])
    else:
        assert np.array_equal(ix.sample_indices0(), z[p + "sample0"])


def test_rms_production_rows(golden_dir):
    """RunningMeanStd at the headline's row count: two updates on [4096, 376] batches of the
    synthetic env's raw rows (regenerated from the env keys) give the reference's f32
    mean / var bit for bit (tools/gen_goldens.py gen_rms_wide; statistics.py:99-114)."""
    z = _load(golden_dir, "rms_wide.npz")
    E, D = int(z["E"]), int(z["D"])
    r = ref.RMS()
    for i in range(2):
        k = synth_env.key(0, np.arange(E), np.zeros(E, np.int64), np.full(E, int(z[f"t{i}"])))
        r.update(synth_env.box_obs(k, D))
        assert np.array_equal(np.asarray(r.mean), z[f"mean{i}"])
        assert np.array_equal(np.asarray(r.var), z[f"var{i}"])
        assert r.count == int(z[f"count{i}"])


def test_synth_env_obs_rms_production_rows(golden_dir):
    """The reference Collector + VectorEnvNormObs at 4096 envs x D = 376 (gen_collector_wide):
    the NumPy env + RMS restatement reproduces obs_rms after the initial reset and after every
    one of the 8 vector steps bit for bit, and the stored rewards."""
    z = _load(golden_dir, "collector_wide.npz")
    E, D, L, T = (int(z[k]) for k in ("E", "D", "L", "T"))
    env = synth_env.SynthVecEnvNP(E, (D,), int(z["A"]), L)
    rms = ref.RMS()

    def check(t):
        assert np.array_equal(np.asarray(rms.mean, np.float32), z[f"rms{t}_mean"]), t
        assert np.array_equal(np.asarray(rms.var, np.float32), z[f"rms{t}_var"]), t
        assert rms.count == int(z[f"rms{t}_count"]), t

    rms.update(env.reset())
    check(0)
    rew = np.zeros((E, T))
    for t in range(T):
        nxt, rew[:, t], term, trunc = env.step()
        rms.update(nxt)
        done = np.flatnonzero(term | trunc)
        if len(done):
            rms.update(env.reset(done))
        check(t + 1)
    assert np.array_equal(rew.reshape(-1), z["c1_rew"])


def test_headline_rows_rebuild_matches_reference(golden_dir):
    """The full-length headline obs_rms trajectory (gen_rms_fullT: the reference
    VectorEnvNormObs over 4096 synthetic envs x 2048 steps, D = 376, L = 1000): the done ids of
    every step follow the env's closed form, the counts add up, the first steps' statistics
    equal the NumPy restatement (ref.RMS over oracle.synth_env rows) bit for bit, and
    oracle.headline.rebuild_rows -- the rows the GPU test compares the device buffer with --
    reproduces every normalised row the reference wrapper returned for the kept envs and steps
    (obs_next, reset rows, initial obs) bit for bit."""
    from oracle import headline
    z = _load(golden_dir, "rms_fullT.npz")
    E, D, L, T = (int(z[k]) for k in ("E", "D", "L", "T"))
    e = np.arange(E)
    cnt = z["counts"]
    assert cnt[0, 0] == E
    for s in range(T):
        _, t = headline.step_coords(e, s, L)
        done = np.flatnonzero(t == L)
        assert np.array_equal(headline.done_ids(z, s), done), s
        prev = cnt[s, 1] if s else cnt[0, 0]  # row 0: the initial reset's update only
        assert cnt[s + 1, 0] == prev + E and cnt[s + 1, 1] == cnt[s + 1, 0] + len(done)
    # the first 3 steps through the NumPy restatement (the env's own step / reset calls)
    env = synth_env.SynthVecEnvNP(E, (D,), int(z["A"]), L)
    rms = ref.RMS()
    rms.update(env.reset())
    assert np.array_equal(np.asarray(rms.mean, np.float32), z["step_mean"][0])
    for s in range(3):
        nxt, _, term, trunc = env.step()
        rms.update(nxt)
        assert np.array_equal(np.asarray(rms.mean, np.float32), z["step_mean"][s + 1])
        assert np.array_equal(np.asarray(rms.var, np.float32), z["step_var"][s + 1])
        done = np.flatnonzero(term | trunc)
        if len(done):
            rms.update(env.reset(done))
        assert np.array_equal(np.asarray(rms.var, np.float32), z["reset_var"][s])
    keep, steps = z["keep_envs"], z["keep_steps"]
    obs, obs_next = headline.rebuild_rows(z, keep)
    assert np.array_equal(obs[:, 0], z["kept_obs0"])
    for i, s in enumerate(steps):
        assert np.array_equal(obs_next[:, s], z["kept_obs_next"][i]), s
    n_reset = 0
    for name in z.files:
        if name.startswith("kept_reset_"):
            s, env_id = (int(v) for v in name.split("_")[2:])
            if s + 1 < T:
                a = int(np.flatnonzero(keep == env_id)[0])
                assert np.array_equal(obs[a, s + 1], z[name]), name
                n_reset += 1
    assert n_reset >= 6


def test_cpu_port_matches_reference_collector(golden_dir):
    """bench.py's cpu_baseline (oracle/cpu_port.py) is a parity-checked restatement: one
    iteration at config 2's width (16 envs x 24 steps, Box 17/6, L = 7) from the reference
    policy's initial weights reproduces the reference Collector + VectorEnvNormObs run of
    collector_d17.npz -- obs_rms and every stored obs / obs_next row and reward bit for bit
    (actions do not enter the synthetic env), and process_fn's V(s), returns and advantages
    (rew_norm GAE, a2c.py:83-117) within north_star's rtol 1e-5, atol 1e-6 * max."""
    from oracle import cpu_port
    z = _load(golden_dir, "collector_d17.npz")
    E, D, A, L, T = (int(z[k]) for k in ("E", "D", "A", "L", "T"))
    init = {k[len("init_"):]: z[k] for k in z.files if k.startswith("init_actor.") or
            k.startswith("init_critic.")}
    rec = {}
    cpu_port.run_iteration(E, T, D, A, repeat=1, minibatches=4, ep_len=L, threads=1,
                           init=init, record=rec)
    assert np.array_equal(rec["rms_mean"].astype(np.float32), z["c1_rms_mean"])
    assert np.array_equal(rec["rms_var"].astype(np.float32), z["c1_rms_var"])
    assert rec["rms_count"] == int(z["c1_rms_count"])
    assert np.array_equal(rec["obs"], z["c1_buf_obs"])
    assert np.array_equal(rec["obs_next"], z["c1_buf_obs_next"])
    assert np.array_equal(rec["rew"], z["c1_buf_rew"])
    for k in ("v_s", "returns", "adv"):
        want = z["pf_" + k]
        np.testing.assert_allclose(rec[k], want, rtol=1e-5, atol=1e-6 * np.abs(want).max(),
                                   err_msg=k)
