"""Flat gradient / Adam storage for one parameter list: every ``.grad`` is a view into one
bucket, and -- when the optimiser is a plain ``torch.optim.Adam`` over exactly these
parameters -- the parameters and their Adam moments become views into flat buffers, so
``clip_grad_norm_`` + ``optim.step()`` (ppo.py:143-151) run as ONE HIP pass
(``tsrl_clip_adam``, csrc/optim.hip) whose learning rate is a device word.  Both properties
make a whole epoch of minibatches capturable as one HIP graph: no host-side optimiser logic,
no allocation, no synchronisation.

``optim.state[p]`` entries are views too, so ``optim.state_dict()`` and torch's own
``optim.step()`` work on the same storage; after ``optim.load_state_dict()`` the next
``adam_bound`` check copies the loaded moments and step counts into the flat storage.

Used by the fused Gaussian MLP (policy/fused_mlp.py, which adds its kernels' pointers) and by
the Categorical learn path of PPOPolicy (any torch actor / critic networks).
"""
from typing import Optional

import torch

from tianshou_amd import _C


def _slot(flat: torch.Tensor, o: int, p: torch.Tensor) -> torch.Tensor:
    """The numel(p) words of ``flat`` from offset o viewed with p's shape AND memory format
    (a channels_last conv weight stays channels_last: MIOpen would otherwise copy an NCHW
    weight to the input's format on every convolution, and autograd would accumulate its
    channels_last gradients into NCHW slots with a strided add)."""
    k = p.numel()
    if p.is_contiguous():
        return flat[o:o + k].view_as(p)
    stride = torch.empty_like(p, memory_format=torch.preserve_format).stride()
    return flat.as_strided(p.shape, stride, flat.storage_offset() + o)


class FlatAdam:
    # extra f32 words after the flat gradients in the bucket (data-parallel loss sums ride
    # in the same all-reduce as the gradients)
    BUCKET_TAIL = 0

    def __init__(self, params) -> None:
        self.params = [p for p in params]
        self._flat = None
        self._bucket = None
        self._views = []
        self._adam = None  # flat parameter / moment storage of bind_adam

    # -- gradient storage -----------------------------------------------------------------------
    def bind_grads(self) -> None:
        """Point every parameter's .grad at a slice of one flat buffer (kept across
        minibatches; re-bound if the optimiser or user replaced a .grad)."""
        dev = self.params[0].device
        if self._flat is not None and all(
                p.grad is not None and p.grad.data_ptr() == v.data_ptr()
                for p, v in zip(self.params, self._views)):
            return
        n = sum(p.numel() for p in self.params)
        self._bucket = torch.zeros(n + self.BUCKET_TAIL, dtype=torch.float32, device=dev)
        self._flat = self._bucket[:n]
        self._views = []
        o = 0
        for p in self.params:
            v = _slot(self._flat, o, p)
            p.grad = v
            self._views.append(v)
            o += p.numel()
        self._grads_bound()

    def _grads_bound(self) -> None:
        """Hook: the gradient addresses changed."""

    @property
    def flat_grad(self) -> Optional[torch.Tensor]:
        return self._flat

    def zero_grad(self) -> None:
        """optim.zero_grad() for views that must keep their addresses: autograd then
        accumulates into the flat bucket in place."""
        self.bind_grads()
        self._flat.zero_()

    def release_grads(self) -> None:
        """zero_grad() for an eager backward followed by gather_grads(): the slots stay bound
        (their addresses are the ones the optimiser pass and the collectives use), every .grad
        is set to None, and autograd then hands each parameter its gradient tensor as it is
        instead of adding it into a zero-filled slot -- the fill and one add per parameter
        saved (round 6; 12 of each per config-5 minibatch)."""
        self.bind_grads()
        for p, v in zip(self.params, self._views):
            p.grad = None
            # a custom backward that can write a gradient in place (net_atari's Flatten +
            # Linear) finds its slot here, writes it and makes it the .grad
            p._tsrl_flat_slot = v

    def gather_grads(self) -> None:
        """After a backward that began with release_grads(): every parameter's gradient copied
        into its slot in one multi-tensor pass (a slot whose parameter received no gradient is
        zeroed, as zero_grad() would have left it) and every .grad pointed back at its slot."""
        dst, src = [], []
        for p, v in zip(self.params, self._views):
            p.__dict__.pop("_tsrl_flat_slot", None)
            g = p.grad
            if g is None:
                v.zero_()
            elif g.data_ptr() != v.data_ptr():
                if g.shape != v.shape or g.dtype != v.dtype:
                    raise RuntimeError("FlatAdam.gather_grads: a gradient does not match its "
                                       f"parameter ({tuple(g.shape)} {g.dtype} vs "
                                       f"{tuple(v.shape)} {v.dtype})")
                dst.append(v)
                src.append(g)
            p.grad = v
        if dst:
            torch._foreach_copy_(dst, src)

    # -- clip_grad_norm_ + Adam as one HIP pass ---------------------------------------------------
    @staticmethod
    def _plain_adam(optim, params) -> bool:
        if not isinstance(optim, torch.optim.Adam) or len(optim.param_groups) != 1:
            return False
        g = optim.param_groups[0]
        if g.get("amsgrad") or g.get("weight_decay", 0) != 0 or g.get("maximize") or \
                g.get("differentiable") or isinstance(g["lr"], torch.Tensor):
            return False
        return len(g["params"]) == len(params) and \
            all(a is b for a, b in zip(g["params"], params))

    def adam_bound(self, optim) -> bool:
        """The flat storage serves ``optim``: same optimiser, parameters still views into the
        flat buffer.  If ``optim.state`` no longer holds the flat views (``load_state_dict``
        installs new exp_avg / exp_avg_sq / step tensors), the loaded moments and step counts
        are copied into the flat storage and the views re-installed, so a restored state is
        what the next clip_adam pass continues from."""
        st = self._adam
        if st is None or st["optim"] is not optim or not all(
                p.data_ptr() == v.data_ptr() for p, v in zip(self.params, st["pviews"])):
            return False
        if not self._state_is_flat(optim):
            if not self._uniform_steps(optim, self.params):
                # a partial / mixed state dict: torch's Adam keeps one step count per
                # parameter, the flat pass one for all -- hand the step back to torch
                self._adam = None
                return False
            self._rebind_state(optim)
        return True

    @staticmethod
    def _uniform_steps(optim, params) -> bool:
        """Every parameter's Adam step count is the same (a parameter without state counts
        0).  clip_adam applies one bias correction to all parameters, so only then is it the
        update torch's Adam would make."""
        ks = set()
        for p in params:
            s = optim.state.get(p, {})
            ks.add(float(s["step"]) if "step" in s else 0.0)
        return len(ks) <= 1

    def _state_is_flat(self, optim) -> bool:
        st = self._adam
        for i, p in enumerate(self.params):
            s = optim.state.get(p)
            if s is None:
                return False
            m, v, k = s.get("exp_avg"), s.get("exp_avg_sq"), s.get("step")
            if not (isinstance(m, torch.Tensor) and isinstance(v, torch.Tensor) and
                    isinstance(k, torch.Tensor)):
                return False
            if m.data_ptr() != st["mviews"][i].data_ptr() or \
                    v.data_ptr() != st["vviews"][i].data_ptr() or \
                    k.data_ptr() != st["steps"][i].data_ptr():
                return False
        return True

    def _rebind_state(self, optim) -> None:
        """Copy whatever ``optim.state`` now holds into the flat moments / step counts (zeros
        for a parameter without state) and point ``optim.state`` back at the flat views."""
        st = self._adam
        for i, p in enumerate(self.params):
            s = optim.state.get(p, {})
            if "exp_avg" in s:
                st["mviews"][i].copy_(s["exp_avg"])
                st["vviews"][i].copy_(s["exp_avg_sq"])
                st["steps"][i].copy_(torch.as_tensor(s["step"], dtype=torch.float32))
            else:
                st["mviews"][i].zero_()
                st["vviews"][i].zero_()
                st["steps"][i].zero_()
            optim.state[p] = {"step": st["steps"][i], "exp_avg": st["mviews"][i],
                              "exp_avg_sq": st["vviews"][i]}
        st["lr_host"] = None  # load_state_dict may also have changed the param-group lr

    def bind_adam(self, optim) -> bool:
        """Move every parameter and its Adam moments into flat buffers (parameter .data and
        ``optim.state[p]`` become views) when ``optim`` is a plain Adam over exactly these
        parameters; then ``clip_adam`` replaces clip_grad_norm_ + optim.step()."""
        if self.adam_bound(optim):
            return True
        if not self._plain_adam(optim, self.params) or not self._uniform_steps(optim, self.params):
            self._adam = None
            return False
        dev = self.params[0].device
        n = sum(p.numel() for p in self.params)
        flat_p = torch.empty(n, dtype=torch.float32, device=dev)
        flat_m = torch.zeros(n, dtype=torch.float32, device=dev)
        flat_v = torch.zeros(n, dtype=torch.float32, device=dev)
        steps = torch.zeros(len(self.params), dtype=torch.float32, device=dev)
        pviews, mviews, vviews = [], [], []
        o = 0
        for i, p in enumerate(self.params):
            k = p.numel()
            pv, mv, vv = _slot(flat_p, o, p), _slot(flat_m, o, p), _slot(flat_v, o, p)
            pv.copy_(p.detach())
            st = optim.state.get(p, {})
            if "exp_avg" in st:
                mv.copy_(st["exp_avg"])
                vv.copy_(st["exp_avg_sq"])
                steps[i] = float(st["step"])
            with torch.no_grad():
                p.data = pv
            optim.state[p] = {"step": steps[i], "exp_avg": mv, "exp_avg_sq": vv}
            pviews.append(p.data)
            mviews.append(optim.state[p]["exp_avg"])
            vviews.append(optim.state[p]["exp_avg_sq"])
            o += k
        self._adam = dict(optim=optim, p=flat_p, m=flat_m, v=flat_v, steps=steps, pviews=pviews,
                          mviews=mviews, vviews=vviews,
                          ticket=torch.zeros(3, dtype=torch.int32, device=dev),
                          partials=torch.zeros(
                              max(int(_C.lib().tsrl_clip_adam_partials(n)), 1),
                              dtype=torch.float64, device=dev),
                          norm=torch.zeros(2, dtype=torch.float32, device=dev),
                          lr=torch.zeros(1, dtype=torch.float32, device=dev))
        self._flat = None  # parameter addresses moved: bind_grads re-derives every pointer
        self.bind_grads()
        return True

    def flat_offset(self, t: torch.Tensor) -> int:
        """Element offset of parameter storage ``t`` inside the flat parameter buffer."""
        return (t.data_ptr() - self._adam["p"].data_ptr()) // 4

    def set_lr(self) -> None:
        """Publish the optimiser's current lr to the device word the Adam kernel reads (one
        tiny fill per epoch; captured learn graphs then follow an lr_scheduler without being
        re-captured)."""
        st = self._adam
        lr = float(st["optim"].param_groups[0]["lr"])
        if st.get("lr_host") != lr:
            st["lr"].fill_(lr)
            st["lr_host"] = lr

    def clip_adam(self, max_norm: Optional[float], scale_grads: bool = True,
                  split=None) -> None:
        """clip_grad_norm_(max_norm) (when given) + Adam.step() over the flat buffers; the
        learning rate comes from the device word of set_lr().  ``scale_grads=False`` skips
        the in-place clipping of .grad (only the last step of a learn() needs it: every
        minibatch overwrites the gradients); ``split`` (a _C.W1Split) re-splits first-layer
        weights into bf16x6 planes in the same pass."""
        st = self._adam
        g = st["optim"].param_groups[0]
        b1, b2 = g["betas"]
        if st.get("lr_host") is None:
            self.set_lr()
        _C.check(_C.lib().tsrl_clip_adam(
            _C.ptr(st["p"]), _C.ptr(self._flat), _C.ptr(st["m"]), _C.ptr(st["v"]),
            st["p"].numel(), _C.ptr(st["steps"]), st["steps"].numel(), float(g["lr"]),
            float(b1), float(b2), float(g["eps"]), float(max_norm) if max_norm else 0.0,
            _C.ptr(st["partials"]), _C.ptr(st["norm"]), _C.ptr(st["ticket"]), _C.ptr(st["lr"]),
            split, int(bool(scale_grads)), _C.stream_ptr(st["p"].device)),
            "tsrl_clip_adam")

    def check_handoff(self) -> None:
        """Raise if any clip_adam launch since the last check timed out waiting for the slice
        norms of the other workgroups (tsrl_clip_adam's sticky ticket[2]): its step used a
        NaN clip coefficient in some slices only, so the parameters are invalid.  One 4-byte
        read, after learn() has read its loss terms back anyway."""
        st = self._adam
        if st is not None and int(st["ticket"][2].item()) != 0:
            st["ticket"][2].zero_()
            raise RuntimeError("tsrl_clip_adam: the in-kernel gradient-norm hand-off timed out "
                               "(workgroups not co-resident); this learn()'s parameters are "
                               "invalid")
