"""ctypes binding of libtsrl.so (include/tsrl.h) -- the only way this package reaches the GPU
kernels.  There is no CPU fallback: if the library is missing, or a tensor handed to a
kernel is not a HIP device tensor, the call raises.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# TSRL_LIB_PATH: load another build of the same library (kernel-variant experiments, tools/)
LIB_PATH = os.environ.get("TSRL_LIB_PATH") or os.path.join(_HERE, "lib", "libtsrl.so")

_i64 = ctypes.c_int64
_u64 = ctypes.c_uint64
_p = ctypes.c_void_p
_d = ctypes.c_double
_f = ctypes.c_float
_i32 = ctypes.c_int32


class AddArgs(ctypes.Structure):
    """Mirror of ``tsrl_add_args`` (field order must match include/tsrl.h)."""
    _fields_ = [
        ("ids", _p), ("ptr", _p), ("next_rel", _p), ("offset", _p), ("k", _i64),
        ("uniform_rel", _i64), ("uniform_next", _i64), ("rel_dev", _p), ("ring_size", _i64),
        ("obs_src", _p), ("obs_dst", _p), ("obs_row_bytes", _i64),
        ("obs_next_src", _p), ("obs_next_dst", _p), ("cur_obs", _p), ("obs_dim", _i64),
        ("norm_mean", _p), ("norm_var", _p), ("norm_eps", _f), ("norm_clip", _f),
        ("obs_next_src_raw", _p), ("obs_next_dst_raw", _p),
        ("act_src", _p), ("act_dst", _p), ("act_row_bytes", _i64),
        ("rew", _p), ("term", _p), ("trunc", _p),
        ("rew_dst", _p), ("term_dst", _p), ("trunc_dst", _p), ("done_dst", _p),
        ("env_id_dst", _p),
        ("ep_rew", _p), ("ep_len", _p), ("ep_idx", _p),
        ("out_ep_rew", _p), ("out_ep_len", _p), ("out_ep_idx", _p),
        ("stat_rew", _p), ("stat_len", _p), ("stat_idx", _p),
        ("reset_src", _p), ("reset_mask", _p), ("reset_mean", _p), ("reset_var", _p),
        ("rel_next", _p), ("obs_src_pitch", _i64), ("obs_next_src_pitch", _i64),
        ("obs_dst_pitch", _i64),
    ]


class CollectArgs(ctypes.Structure):
    """Mirror of ``tsrl_collect_args`` (field order must match include/tsrl.h)."""
    _fields_ = [
        ("add", AddArgs), ("k", _i64), ("dim", _i64), ("cur", _p),
        ("obs_dst", _p), ("obs_offset", _p), ("obs_rel_dev", _p), ("obs_uniform_rel", _i64),
        ("w1p", _p), ("b1", _p), ("w2", _p), ("b2", _p), ("w3", _p), ("b3", _p),
        ("log_std", _p), ("act_dim", _i64), ("act_seed", _u64), ("rng_ctr", _p),
        ("rng_next", _p), ("sample", _i32), ("bound_method", _i32), ("low", _p), ("high", _p),
        ("act", _p), ("act_remap", _p),
        ("env_seed", _u64), ("ep_len", _i64), ("ep_j", _p), ("ep_t", _p),
        ("raw", _p), ("reset_raw", _p), ("rew", _p), ("term", _p), ("trunc", _p), ("done", _p),
        ("workspace", _p), ("mean", _p), ("var", _p), ("snap_mean", _p), ("snap_var", _p),
        ("count", _p), ("no_moments", _i64), ("rms_step", _i64), ("obs_pitch", _i64),
        ("act_coef", ctypes.c_float),
        ("xpipe", _i64), ("xstats", _p), ("spec_j", _p), ("spec_t", _p), ("spec_raw", _p),
        ("spec_reset_raw", _p), ("spec_done", _p),
    ]


class PPOParams(ctypes.Structure):
    """Mirror of ``tsrl_ppo_params``."""
    _fields_ = [
        ("eps_clip", _d), ("dual_clip", _d), ("vf_coef", _d), ("ent_coef", _d),
        ("adv_eps", _d), ("b_global", _d), ("value_clip", _i32), ("norm_adv", _i32),
    ]


class TailWeights(ctypes.Structure):
    """Mirror of ``tsrl_tail_weights``."""
    _fields_ = [(k, _p) for k in ("w2a", "b2a", "w2c", "b2c", "w3a", "b3a", "w3c", "b3c",
                                  "log_std")]


class W1Split(ctypes.Structure):
    """Mirror of ``tsrl_w1_split``."""
    _fields_ = [("out", _p), ("off_a", _i64), ("off_c", _i64), ("d", _i64), ("kp", _i64)]


class TailGrads(ctypes.Structure):
    """Mirror of ``tsrl_tail_grads``."""
    _fields_ = [(k, _p) for k in ("w2a", "b2a", "w2c", "b2c", "w3a", "b3a", "w3c", "b3c")]


_SIGS = {
    "tsrl_version": ([], ctypes.c_char_p),
    "tsrl_last_error": ([], ctypes.c_char_p),
    "tsrl_gae_workspace_bytes": ([_i64, _i64], _i64),
    "tsrl_gae_num_partials": ([_i64, _i64], _i64),
    "tsrl_gae_time_next": ([_p, _p], ctypes.c_int),
    "tsrl_gae": ([_p, _p, _p, _p, _p, _p, _i64, _i64, _p, _d, _d, _p, _p, _p, _p, _p, _p, _i64,
                  _p], ctypes.c_int),
    "tsrl_gae_f64v": ([_p, _p, _p, _p, _p, _p, _i64, _i64, _d, _d, _p, _p, _p, _i64, _p],
                      ctypes.c_int),
    "tsrl_ret_rms_update": ([_p, _i64, _p, _p], ctypes.c_int),
    "tsrl_env_num_partials": ([_i64], _i64),
    "tsrl_synth_box_step": ([_p, _i64, _i64, _u64, _i64, _p, _p, _p, _p, _p, _p, _p, _p],
                            ctypes.c_int),
    "tsrl_synth_box_step_reset": ([_i64, _i64, _u64, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                                   _p, _p, _p], ctypes.c_int),
    "tsrl_synth_box_step_act": ([_p, _i64, _i64, _u64, _i64, _p, _p, _p, _p, _p, _p, _p, _p,
                                 _i64, ctypes.c_float, _p], ctypes.c_int),
    "tsrl_synth_box_step_reset_act": ([_i64, _i64, _u64, _i64, _p, _p, _p, _p, _p, _p, _p, _p,
                                       _p, _p, _p, _p, _i64, ctypes.c_float, _p],
                                      ctypes.c_int),
    "tsrl_rms_merge2": ([_p, _p, _p, _i64, _i64, _i64, _p, _p, _p, _p, _p, _p, _p, _p],
                        ctypes.c_int),
    "tsrl_synth_box_reset": ([_p, _p, _i64, _i64, _u64, _i64, _p, _p, _p, _p, _p], ctypes.c_int),
    "tsrl_synth_u8_step": ([_p, _i64, _i64, _i64, _u64, _i64, _p, _p, _p, _p, _p, _p, _p],
                           ctypes.c_int),
    "tsrl_synth_u8_reset": ([_p, _p, _i64, _i64, _i64, _u64, _i64, _p, _p, _p, _p],
                            ctypes.c_int),
    "tsrl_cartpole_step": ([_p, _i64, _p, _i64, _p, _p, _p, _p, _p, _p, _p], ctypes.c_int),
    "tsrl_cartpole_reset": ([_p, _p, _i64, _u64, _p, _p, _p, _p, _p], ctypes.c_int),
    "tsrl_rms_merge": ([_p, _i64, _i64, _p, _i64, _p, _p, _p, _p, _p, _p], ctypes.c_int),
    "tsrl_rms_sum_partials2": ([_p, _p, _p, _i64, _i64, _i64, _p, _p], ctypes.c_int),
    "tsrl_rms_norm_rows": ([_p, _p, _i64, _i64, _p, _p, _f, _f, _p, _p], ctypes.c_int),
    "tsrl_buffer_add": ([ctypes.POINTER(AddArgs), _p], ctypes.c_int),
    "tsrl_ring_advance": ([_p, _i64, _p], ctypes.c_int),
    "tsrl_collect_pack_floats": ([_i64], _i64),
    "tsrl_collect_pack_w1": ([_p, _i64, _p, _p], ctypes.c_int),
    "tsrl_collect_workspace_bytes": ([_i64, _i64], _i64),
    "tsrl_collect_box_step": ([ctypes.POINTER(CollectArgs), _p], ctypes.c_int),
    "tsrl_collect_rms_finalize": ([ctypes.POINTER(CollectArgs), _p], ctypes.c_int),
    "tsrl_collect_totals_offset": ([_i64], _i64),
    "tsrl_collect_spec_step": ([ctypes.POINTER(CollectArgs), _i32, _p], ctypes.c_int),
    "tsrl_collect_xpipe_finalize": ([ctypes.POINTER(CollectArgs), _p], ctypes.c_int),
    "tsrl_rms_exact_stats_bytes": ([_i64], _i64),
    "tsrl_rms_exact_stats": ([_p, _i64, _p, _p, _i64, _p, _p], ctypes.c_int),
    "tsrl_rms_exact_stats_n": ([_i32, _p, _p, _p, _i64, _i64, _p, _p], ctypes.c_int),
    "tsrl_rms_exact_stats_max_steps": ([], ctypes.c_int),
    "tsrl_gather_rows": ([_p, _i64, _p, _i64, _p, _p], ctypes.c_int),
    "tsrl_gather_rows_pitched": ([_p, _i64, _i64, _p, _i64, _p, _p], ctypes.c_int),
    "tsrl_np_shuffle_draws": ([_p, _p, _i64, _p], ctypes.c_int),
    "tsrl_shuffle_apply_workspace_bytes": ([_i64], _i64),
    "tsrl_shuffle_apply": ([_p, _i64, _p, _p, _i64, _p], ctypes.c_int),
    "tsrl_ring_step_index": ([_p, _i64, _p, _p, _p, _i64, _i64, ctypes.c_int, _p, _p],
                             ctypes.c_int),
    "tsrl_stack_gather_pitched": ([_p, _i64, _i64, _p, _i64, _i64, _p, _p, _p, _i64, _i64, _p,
                                   _p, _p], ctypes.c_int),
    "tsrl_stack_gather": ([_p, _i64, _p, _i64, _i64, _p, _p, _p, _i64, _i64, _p, _p, _p],
                          ctypes.c_int),
    "tsrl_frames_to_f32_nhwc": ([_p, _i64, _i64, _i64, _p, _p, _p], ctypes.c_int),
    "tsrl_dqn_conv1_fwd": ([_p, _i64, _p, _p, _i64, _i64, _i64, _i64, _p, _f, ctypes.c_int, _p,
                            _p],
                           ctypes.c_int),
    "tsrl_dqn_conv2_dgrad": ([_p, _i64, _p, _i64, _i64, _i64, _i64, _p, _p, _p], ctypes.c_int),
    "tsrl_relu_bwd_rows_workspace_bytes": ([_i64, _i64], _i64),
    "tsrl_relu_bwd_rows": ([_p, _p, _p, _i64, _i64, _p, _p, _i64, _p], ctypes.c_int),
    "tsrl_bias_relu_rows": ([_p, _p, _i64, _i64, _p], ctypes.c_int),
    "tsrl_dqn_conv1_wgrad_workspace_bytes": ([_i64], _i64),
    "tsrl_dqn_conv1_wgrad": ([_p, _i64, _p, _p, _f, _p, _p, _p, _i64, _p], ctypes.c_int),
    "tsrl_nstep_return": ([_p, _p, _p, _p, _p, _i64, _i64, _p, _i64, _i64, _d, _p, _i64,
                           ctypes.c_int, _p, _p], ctypes.c_int),
    "tsrl_clip_adam_partials": ([_i64], _i64),
    "tsrl_clip_adam": ([_p, _p, _p, _p, _i64, _p, _i64, _f, _f, _f, _f, _f, _p, _p, _p, _p,
                        ctypes.POINTER(W1Split), ctypes.c_int, _p],
                       ctypes.c_int),
    "tsrl_segtree_set": ([_p, _i64, _p, _p, _i64, _i64, _p, _p], ctypes.c_int),
    "tsrl_segtree_reduce": ([_p, _i64, _i64, _i64, _p, _p], ctypes.c_int),
    "tsrl_segtree_prefix_idx": ([_p, _i64, _p, ctypes.c_int, _i64, _p, _p], ctypes.c_int),
    "tsrl_sum_rows_workspace_bytes": ([_i64, _i64], _i64),
    "tsrl_sum_rows_f32": ([_p, _i64, _i64, _p, _p, _i64, _p], ctypes.c_int),
    "tsrl_ppo_num_partials": ([_i64], _i64),
    "tsrl_adv_moments": ([_p, _p, _i64, _p, _p], ctypes.c_int),
    "tsrl_reduce_partials": ([_p, _i64, _i64, _p, _p], ctypes.c_int),
    "tsrl_adv_moments_seg_parts": ([_i64], _i64),
    "tsrl_adv_moments_seg": ([_p, _p, _p, _i64, _i64, _p, _p, _p], ctypes.c_int),
    "tsrl_ppo_gauss_fwd_bwd": ([_p, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, _p, PPOParams,
                                _p, _p, _p, _p], ctypes.c_int),
    "tsrl_ppo_gauss_finalize": ([_p, _i64, _p, PPOParams, _p, _p, _p], ctypes.c_int),
    "tsrl_gauss_logp": ([_p, _p, _p, _i64, _i64, _p, _p], ctypes.c_int),
    "tsrl_ppo_cat_fwd_bwd": ([_p, _p, _p, _p, _p, _p, _p, _p, _i64, _i64, ctypes.c_int, _p,
                              PPOParams, _p, _p, _p, _p], ctypes.c_int),
    "tsrl_ppo_cat_finalize": ([_p, PPOParams, _p, _p], ctypes.c_int),
    "tsrl_cat_logp": ([_p, _p, _i64, _i64, ctypes.c_int, _p, _p], ctypes.c_int),
    "tsrl_cat_gumbel_argmax": ([_p, _p, _i64, _i64, _p, _p], ctypes.c_int),
    "tsrl_rms_exact_update": ([_p, _p, _i64, _p, _p, _i64, _i64, _p, _p, _p, _p, _p, _p, _p],
                              ctypes.c_int),
    "tsrl_np_shuffle_draws_mt": ([_p, _p, _i64, _p, ctypes.c_int], ctypes.c_int),
    "tsrl_mlp_l1_fwd": ([_p, _i64, _p, _i64, _i64, _p, _p, _p, _p, ctypes.c_int, _p,
                         ctypes.c_int, _p], ctypes.c_int),
    "tsrl_mlp_frag_floats": ([_i64], _i64),
    "tsrl_mlp_split_bytes": ([_i64], _i64),
    "tsrl_mlp_split_w": ([_p, _p, _i64, _p, _p], ctypes.c_int),
    "tsrl_mlp_l1_fwd_x6": ([_p, _i64, _p, _i64, _i64, _p, _p, _p, ctypes.c_int, _p,
                            ctypes.c_int, _p], ctypes.c_int),
    "tsrl_ppo_tail_workspace_bytes": ([_i64], _i64),
    "tsrl_ppo_tail": ([_p, _i64, _p, ctypes.POINTER(TailWeights), _i64, _p, _p, _p, _p, _p, _p,
                       PPOParams, _p, ctypes.POINTER(TailGrads), _p, _p, _i64, _p],
                      ctypes.c_int),
    "tsrl_ppo_tail_fin": ([_p, _i64, _p, ctypes.POINTER(TailWeights), _i64, _p, _p, _p, _p, _p,
                           _p, PPOParams, _p, ctypes.POINTER(TailGrads), _p, _p, _i64, _p, _p,
                           _p, _p], ctypes.c_int),
    "tsrl_ppo_tail_stage": ([_p, _i64, _p, ctypes.POINTER(TailWeights), _i64, _p, _p, _p, _p,
                             _p, _p, PPOParams, _p, ctypes.POINTER(TailGrads), _p, _p, _i64, _p,
                             _p, _p, ctypes.c_int, _p], ctypes.c_int),
    "tsrl_ppo_eval": ([_p, _i64, ctypes.POINTER(TailWeights), _i64, _p, _p, _p, _p],
                      ctypes.c_int),
    "tsrl_ppo_eval_fused_workspace_bytes": ([], _i64),
    "tsrl_ppo_eval_fused": ([_p, _i64, _p, _i64, _i64, _p, _p, _p, ctypes.POINTER(TailWeights),
                             _i64, _p, _p, _p, _p, _i64, _p], ctypes.c_int),
    "tsrl_mlp_dw_workspace_bytes": ([_i64, _i64], _i64),
    "tsrl_policy_pack_floats": ([_i64], _i64),
    "tsrl_gauss_policy_act_rng": ([_p, _i64, _i64, _i64, _p, _p, _p, _p, _p, _p, _p, _i64, _u64,
                                   _p, _p, ctypes.c_int, _p, _p, _p, _p, _p], ctypes.c_int),
    "tsrl_policy_pack_l1": ([_p, _i64, _p, _p], ctypes.c_int),
    "tsrl_gauss_policy_act": ([_p, _i64, _i64, _i64, _p, _p, _p, _p, _p, _p, _p, _i64, _p,
                               ctypes.c_int, _p, _p, _p, _p, _p], ctypes.c_int),
    "tsrl_mlp_dw": ([_p, _p, _i64, _p, _i64, _i64, _p, _p, _p, _p, _p, _i64, _p], ctypes.c_int),
}

EXPORTED = tuple(_SIGS)
_LIB = None


class TsrlError(RuntimeError):
    pass


def lib():
    """Load libtsrl.so; raise ImportError (loudly) when it has not been built."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libtsrl.so not found at {LIB_PATH}: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _LIB = L
    return _LIB


def check(rc, what=""):
    if rc != 0:
        msg = lib().tsrl_last_error().decode(errors="replace")
        raise TsrlError(f"{what or 'libtsrl'} failed (hipError {rc}): {msg}")


def stream_ptr(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t, dtype=None):
    """Device pointer of a contiguous HIP tensor (None -> NULL)."""
    if t is None:
        return None
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"expected a torch.Tensor, got {type(t)}")
    if t.device.type != "cuda":
        raise TsrlError(f"libtsrl kernels need HIP device tensors; got a tensor on {t.device}")
    if dtype is not None and t.dtype != dtype:
        raise TypeError(f"expected dtype {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError("libtsrl kernels need contiguous tensors")
    return t.data_ptr()


def ptr_rows(t):
    """Device pointer of a HIP tensor whose ROWS are contiguous, the rows possibly further
    apart than their length (a padded storage view [n, d] of [n, pitch]; the caller passes
    the pitch, ``t.stride(0)``, to the kernel)."""
    if t is None:
        return None
    if t.dim() >= 2 and t[0].is_contiguous() and t.stride(0) >= t[0].numel():
        if t.device.type != "cuda":
            raise TsrlError(f"libtsrl kernels need HIP device tensors; got a tensor on {t.device}")
        return t.data_ptr()
    return ptr(t)
