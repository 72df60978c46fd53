"""Device-resident vector envs.

``DeviceVectorEnv`` is the BaseVectorEnv surface (tianshou/env/venvs.py:260-381:
``len``, ``reset(id)``, ``step(action, id)``, ``action_space``/``observation_space``,
``is_async``) with tensors that stay in HBM.  The Collector's fused path additionally calls
``_step_raw``/``_reset_raw``, which write into caller buffers and emit the column partials
that VectorEnvNormObs folds into its running statistics.

``SyntheticVectorEnv`` is the counter-hash env of SURVEY.md §8d, computed by the
``tsrl_synth_*`` kernels (oracle/synth_env.py is its CPU restatement).
"""
from typing import Optional

import numpy as np
import torch

from tianshou_amd import _C
from tianshou_amd.env.spaces import Box, Discrete


class DeviceVectorEnv:
    is_async = False

    def __len__(self) -> int:
        return self.env_num

    def close(self) -> None:
        pass

    def seed(self, seed=None):
        return [seed] * self.env_num

    def _ids(self, id):
        if id is None:
            return None, self.env_num
        ids = np.atleast_1d(np.asarray(id, dtype=np.int64))
        return torch.as_tensor(ids, device=self.device), len(ids)

    def reset(self, id=None, **kwargs):
        ids, k = self._ids(id)
        obs = self.alloc_obs(k)
        self._reset_raw(ids, None, k, obs, None)
        env_id = ids if ids is not None else torch.arange(k, device=self.device)
        return obs, {"env_id": env_id}


class SyntheticVectorEnv(DeviceVectorEnv):
    """Box(obs_dim) f32 or u8 (e.g. 4x84x84) observations, Box(act_dim) or Discrete actions;
    episode length ``ep_len``; even envs terminate, odd envs truncate; actions are ignored
    unless ``act_coef`` is set."""

    def __init__(self, num_envs: int, obs_shape, act_dim: int = 1, ep_len: int = 1000,
                 seed: int = 0, device=None, obs_dtype=np.float32, discrete: bool = False,
                 frame_stack: int = 1, act_coef: float = 0.0):
        """``frame_stack`` S > 1 (u8 only): obs_shape = (S, *frame) holds the last S frames
        like gymnasium's FrameStack wrapper (the Atari setup of
        examples/atari/atari_wrapper.py), so a save_only_last_obs buffer rebuilds it.
        ``act_coef`` c != 0 (Box f32 obs and actions only): the env reads its action, as a
        MuJoCo env does -- a step's observation is f32(box + f32(c * a[d mod act_dim])) of
        the remapped action a (csrc/synth.h coupled_val).  Its observations are then not
        2^-23-quantised and its transition depends on the action, so the fused collect step
        runs the env after the actor and sums obs_rms moments in f64."""
        self.env_num = int(num_envs)
        self.obs_shape = tuple(np.atleast_1d(obs_shape).tolist())
        self.obs_numel = int(np.prod(self.obs_shape))
        self.u8 = np.dtype(obs_dtype) == np.uint8
        self.frame_stack = int(frame_stack)
        assert self.frame_stack == 1 or (self.u8 and self.obs_shape[0] == self.frame_stack), \
            "frame_stack needs u8 observations of shape (frame_stack, ...)"
        self.ep_len, self.seed_ = int(ep_len), int(seed)
        self.device = torch.device(device) if device is not None else \
            torch.device("cuda", torch.cuda.current_device())
        if self.u8:
            self.observation_space = Box(0, 255, self.obs_shape, np.uint8)
        else:
            self.observation_space = Box(-np.inf, np.inf, self.obs_shape, np.float32)
        self.action_space = Discrete(act_dim) if discrete else Box(-1.0, 1.0, (act_dim,))
        self.ep_j = torch.full((self.env_num,), -1, dtype=torch.int64, device=self.device)
        self.ep_t = torch.zeros(self.env_num, dtype=torch.int64, device=self.device)
        self.obs_torch_dtype = torch.uint8 if self.u8 else torch.float32
        self.nblk = int(_C.lib().tsrl_env_num_partials(self.env_num))
        self.act_coef = float(act_coef)
        self.act_dim = int(act_dim)
        assert self.act_coef == 0.0 or (not self.u8 and not discrete), \
            "act_coef needs Box observations and Box actions"

    def _act_arg(self, action, k: int):
        """(pointer, act_dim) of the f32 [k, act_dim] action rows the coupled env reads."""
        if self.act_coef == 0.0:
            return None, 1
        assert action is not None, "the action-coupled env needs the step's actions"
        a = torch.as_tensor(action, device=self.device, dtype=torch.float32)
        a = a.reshape(k, self.act_dim).contiguous()
        self._act_keep = a  # alive until the launch is enqueued (and graph replays)
        return _C.ptr(a), self.act_dim

    # -- fused hooks ---------------------------------------------------------------------------
    def nblk_for(self, k: int) -> int:
        return int(_C.lib().tsrl_env_num_partials(k))

    def alloc_obs(self, k: int) -> torch.Tensor:
        return torch.empty((k,) + self.obs_shape, dtype=self.obs_torch_dtype, device=self.device)

    def alloc_partials(self, k: int) -> Optional[torch.Tensor]:
        if self.u8:
            return None
        n = int(_C.lib().tsrl_env_num_partials(k))
        return torch.empty((n, self.obs_numel, 2), dtype=torch.float64, device=self.device)

    def _step_raw(self, ids: Optional[torch.Tensor], k: int, obs_out, rew_out, term_out,
                  trunc_out, partials=None, action=None) -> None:
        L = _C.lib()
        s = _C.stream_ptr(self.device)
        if self.u8:
            _C.check(L.tsrl_synth_u8_step(_C.ptr(ids), k, self.obs_numel, self.frame_stack,
                                          self.seed_,
                                          self.ep_len, _C.ptr(self.ep_j), _C.ptr(self.ep_t),
                                          _C.ptr(obs_out), _C.ptr(rew_out), _C.ptr(term_out),
                                          _C.ptr(trunc_out), s), "tsrl_synth_u8_step")
        else:
            ap, ad = self._act_arg(action, k)
            _C.check(L.tsrl_synth_box_step_act(_C.ptr(ids), k, self.obs_numel, self.seed_,
                                               self.ep_len, _C.ptr(self.ep_j), _C.ptr(self.ep_t),
                                               _C.ptr(obs_out), _C.ptr(rew_out), _C.ptr(term_out),
                                               _C.ptr(trunc_out), _C.ptr(partials), ap, ad,
                                               self.act_coef, s), "tsrl_synth_box_step")

    @property
    def supports_step_reset(self) -> bool:
        return not self.u8

    def _step_reset_raw(self, k: int, obs_out, reset_out, rew_out, term_out, trunc_out,
                        done_out, partials=None, partials_reset=None, blk_done=None,
                        action=None) -> None:
        """Step all k envs and reset the finished ones in one launch (f32 obs only)."""
        ap, ad = self._act_arg(action, k)
        _C.check(_C.lib().tsrl_synth_box_step_reset_act(
            k, self.obs_numel, self.seed_, self.ep_len, _C.ptr(self.ep_j), _C.ptr(self.ep_t),
            _C.ptr(obs_out), _C.ptr(reset_out), _C.ptr(rew_out), _C.ptr(term_out),
            _C.ptr(trunc_out), _C.ptr(done_out), _C.ptr(partials), _C.ptr(partials_reset),
            _C.ptr(blk_done), ap, ad, self.act_coef, _C.stream_ptr(self.device)),
            "tsrl_synth_box_step_reset")

    def _reset_raw(self, ids: Optional[torch.Tensor], mask: Optional[torch.Tensor], k: int,
                   obs_out, partials=None) -> None:
        """Reset the rows selected by mask (all k without one) into obs_out.  Rows not
        selected are left untouched -- the fused collector relies on it for uint8 obs, whose
        resets are written straight into its current observations."""
        L = _C.lib()
        s = _C.stream_ptr(self.device)
        if self.u8:
            _C.check(L.tsrl_synth_u8_reset(_C.ptr(ids), _C.ptr(mask), k, self.obs_numel,
                                           self.frame_stack, self.seed_, self.ep_len, _C.ptr(self.ep_j),
                                           _C.ptr(self.ep_t), _C.ptr(obs_out), s),
                     "tsrl_synth_u8_reset")
        else:
            _C.check(L.tsrl_synth_box_reset(_C.ptr(ids), _C.ptr(mask), k, self.obs_numel,
                                            self.seed_, self.ep_len, _C.ptr(self.ep_j),
                                            _C.ptr(self.ep_t), _C.ptr(obs_out),
                                            _C.ptr(partials), s), "tsrl_synth_box_reset")

    # -- BaseVectorEnv surface ----------------------------------------------------------------
    def step(self, action, id=None):
        ids, k = self._ids(id)
        obs = self.alloc_obs(k)
        rew = torch.empty(k, dtype=torch.float64, device=self.device)
        term = torch.empty(k, dtype=torch.bool, device=self.device)
        trunc = torch.empty(k, dtype=torch.bool, device=self.device)
        self._step_raw(ids, k, obs, rew, term, trunc, None, action)
        env_id = ids if ids is not None else torch.arange(k, device=self.device)
        return obs, rew, term, trunc, {"env_id": env_id}
