"""Fused Adam on the HIP kernel (GLI:529-530; torch/optim/adam.py _single_tensor_adam).

A drop-in for ``torch.optim.Adam(params, lr, betas, weight_decay)`` as the reference
uses it: the same param_groups and per-parameter state layout
(``state[p] = {step, exp_avg, exp_avg_sq}``), so ``state_dict()`` / ``load_state_dict()``
and ``torch.optim.lr_scheduler.ExponentialLR`` (GLI:533-534, 713-714) work unchanged.
One launch updates every tensor of a param group (multi-tensor, a size-proportional
grid of 4096-element blocks or 32 x 32 x 16 weight bricks, float4 loads, 28 B/element of
HBM traffic) and writes the cached GEMM layouts of the updated weights from the values it
holds (rgan_adam_packed: +4 B/element per layout, no repack pass re-reading the weights).  Hyper-parameters live in a
device buffer (doubles, as torch keeps them in Python floats), refreshed only when a
group's values change; the step counter is a device scalar incremented by the kernel.
"""

import torch
from torch.autograd.graph import increment_version

from . import kernels as K

class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False):
        if amsgrad:
            raise ValueError("amsgrad is not used by the reference and not implemented")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=None,
                        decoupled_weight_decay=False)
        super().__init__(params, defaults)
        self._dev = {}  # group index -> (hyper tensor, host key, step tensor)

    def _group_dev(self, gi, group, device, first_state):
        key = (float(group["lr"]), float(group["betas"][0]), float(group["betas"][1]), float(group["eps"]),
               float(group["weight_decay"]))
        cur = self._dev.get(gi)
        if cur is None or cur[0].device != device:
            hyper = torch.tensor(list(key) + [0.0, 0.0, 0.0], dtype=torch.float64).to(device, non_blocking=True)
            step0 = float(first_state["step"]) if first_state is not None and "step" in first_state else 0.0
            # [count, arrival ticket] (rgan_adam_packed); the count is the 1-element view
            step = torch.tensor([step0, 0.0], dtype=torch.float32).to(device)[:1]
            cur = (hyper, key, step)
            self._dev[gi] = cur
        elif cur[1] != key:
            cur[0].copy_(torch.tensor(list(key) + [0.0, 0.0, 0.0], dtype=torch.float64), non_blocking=True)
            cur = (cur[0], key, cur[2])
            self._dev[gi] = cur
        return cur

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            ps, gs, ms, vs = [], [], [], []
            first = None
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if len(st) and st["exp_avg"].shape != p.shape:
                    raise ValueError(f"Adam state shape {tuple(st['exp_avg'].shape)} != parameter {tuple(p.shape)}")
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                if first is None:
                    first = st
                for k in ("exp_avg", "exp_avg_sq"):
                    if st[k].stride() != p.stride():  # e.g. state loaded from a checkpoint
                        st[k] = torch.empty_like(p).copy_(st[k])
                g = p.grad
                if g.stride() != p.stride():
                    # the kernel walks p, g, m, v with one flat index: g must share p's layout
                    g = g.contiguous() if p.is_contiguous() else torch.empty_like(p).copy_(g)
                ps.append(p)
                gs.append(g)
                ms.append(st["exp_avg"])
                vs.append(st["exp_avg_sq"])
            if not ps:
                continue
            hyper, _, step = self._group_dev(gi, group, ps[0].device, first)
            # one device step counter per group: every stepped parameter must agree with it
            # (torch keeps one per parameter; a parameter that skipped steps would diverge)
            steps = {float(self.state[p]["step"]) for p in ps}
            if len(steps) != 1:
                raise RuntimeError(f"Adam: parameters of group {gi} are at different steps {sorted(steps)}; "
                                   "the fused kernel keeps one step count per group")
            # the kernel also rewrites every cached GEMM layout of these weights from the new values
            layouts = K.PACKS.layouts_of(ps)
            K.adam_packed(ps, gs, ms, vs, hyper, step, layouts)
            for p in ps:
                self.state[p]["step"] += 1  # host mirror of state['step'] (torch Adam's state_dict layout)
                increment_version(p)        # the kernel wrote p: layouts not listed above are stale
            K.PACKS.mark_current(layouts)
        return loss

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._dev = {}
        # torch matches optimizer state to parameters by POSITION and does not check shapes;
        # the kernel trusts p.numel() for exp_avg/exp_avg_sq, so a mismatch must stop here
        for group in self.param_groups:
            for p in group["params"]:
                st = self.state.get(p)
                if not st:
                    continue
                for k in ("exp_avg", "exp_avg_sq"):
                    if k in st and tuple(st[k].shape) != tuple(p.shape):
                        raise ValueError(f"optimizer state '{k}' of shape {tuple(st[k].shape)} does not match its "
                                         f"parameter {tuple(p.shape)} (parameter order differs from the checkpoint)")
