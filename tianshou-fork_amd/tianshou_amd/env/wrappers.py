"""VectorEnvNormObs on device (tianshou/env/venv_wrappers.py:65-112): the running statistics
(obs_rms) are updated with the RAW obs of every step/reset, then the obs are normalised with
the updated statistics and clipped to +-10."""
import torch

from tianshou_amd.utils.statistics import DeviceRunningMeanStd


class VectorEnvNormObs:
    is_async = False

    def __init__(self, venv, update_obs_rms: bool = True, exact_obs_rms: bool = False) -> None:
        """``exact_obs_rms`` (build option, default off): obs_rms with the reference's f32
        arithmetic bit for bit (DeviceRunningMeanStd(exact=True)) instead of f64 moments."""
        self.venv = venv
        self.update_obs_rms = update_obs_rms
        dim = int(getattr(venv, "obs_numel"))
        self.obs_rms = DeviceRunningMeanStd(dim, venv.device, exact=exact_obs_rms)

    def __len__(self) -> int:
        return len(self.venv)

    def __getattr__(self, key):
        if key == "venv":
            raise AttributeError(key)
        return getattr(self.venv, key)

    def reset(self, id=None, **kwargs):
        obs, info = self.venv.reset(id, **kwargs)
        flat = obs.reshape(len(obs), -1).float()
        if self.obs_rms and self.update_obs_rms:
            self.obs_rms.update(flat)
        return self.obs_rms.norm(flat).reshape(obs.shape), info

    def step(self, action, id=None):
        obs, rew, term, trunc, info = self.venv.step(action, id)
        flat = obs.reshape(len(obs), -1).float()
        if self.obs_rms and self.update_obs_rms:
            self.obs_rms.update(flat)
        return self.obs_rms.norm(flat).reshape(obs.shape), rew, term, trunc, info

    def set_obs_rms(self, obs_rms) -> None:
        if isinstance(obs_rms, DeviceRunningMeanStd):
            self.obs_rms = obs_rms
        else:  # host RunningMeanStd (e.g. loaded from a reference checkpoint)
            self.obs_rms.load(obs_rms.mean, obs_rms.var, obs_rms.count)

    def get_obs_rms(self):
        return self.obs_rms
