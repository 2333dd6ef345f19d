"""Fused multi-tensor AdamW (one HIP launch per step for all parameters).

Semantics of torch.optim.AdamW as configured by the reference
(synth_sod/.../lightning_module.py:183-193): weight_decay=0.05, betas=(0.9, 0.999), eps=1e-8,
two param groups (encoder lr, seg_head lr*10).  Parameters whose ``.grad`` is None are skipped
(no decay, no step count change for them), like torch.  LR schedulers work unchanged because
each group's ``lr`` is re-read every step.
"""
from __future__ import annotations

import torch

from ._lib import lib, stream

CHUNK = 65536


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.05):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._tab = None
        self._tab_key = None

    def _table(self, items, dev, step, beta1, wd):
        key = tuple((p.data_ptr(), p.grad.data_ptr() if p.grad is not None else 0,
                     self.state[p]["exp_avg"].data_ptr(), self.state[p]["exp_avg_sq"].data_ptr()) for p, _ in items)
        bc1 = 1.0 - beta1 ** step                 # Python doubles, rounded to f32 once (as torch)
        coef = torch.tensor([[1.0 - g["lr"] * wd, g["lr"] / bc1] for _, g in items], dtype=torch.float32)
        if key != self._tab_key:
            ptrs, sizes, ct, co = [], [], [], []
            for t, (p, g) in enumerate(items):
                st = self.state[p]
                ptrs.append([p.data_ptr(), p.grad.data_ptr() if p.grad is not None else 0,
                             st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()])
                n = p.numel()
                sizes.append(n)
                for o in range(0, n, CHUNK):
                    ct.append(t); co.append(o)
            self._tab = dict(ptrs=torch.tensor(ptrs, dtype=torch.int64, device=dev),
                             sizes=torch.tensor(sizes, dtype=torch.int64, device=dev),
                             ct=torch.tensor(ct, dtype=torch.int32, device=dev),
                             co=torch.tensor(co, dtype=torch.int64, device=dev), n=len(ct))
            self._tab_key = key
        self._tab["coef"] = coef.to(dev, non_blocking=True)
        return self._tab

    def load_state_dict(self, state_dict):
        """torch.optim.AdamW-compatible state (the device pointer table is rebuilt)."""
        super().load_state_dict(state_dict)
        self._tab, self._tab_key = None, None

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        # group parameters by (betas, eps, wd) and shared step count
        items = []
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    # torch.optim.AdamW layout (step as a float tensor) so state_dicts interchange
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                if not torch.is_tensor(st["step"]):
                    st["step"] = torch.tensor(float(st["step"]))
                st["step"] += 1
                items.append((p, g))
        if not items:
            return loss
        steps = {int(self.state[p]["step"].item()) for p, _ in items}
        hyper = {(g["betas"], g["eps"], g["weight_decay"]) for _, g in items}
        if len(steps) != 1 or len(hyper) != 1:
            raise NotImplementedError("FusedAdamW: all stepped parameters must share step count and betas/eps/wd")
        (b1, b2), eps, wd = hyper.pop()
        dev = items[0][0].device
        step = steps.pop()
        tab = self._table(items, dev, step, b1, wd)
        lib()("s3od_adamw_step", tab["ptrs"], tab["sizes"], tab["coef"], tab["ct"], tab["co"], tab["n"], CHUNK,
              step, float(b1), float(b2), float(eps), stream())
        # the kernel writes the masters through raw pointers: bump their version counters so
        # every consumer keyed on `_version` (DPTEngine's packed-weight cache) sees the update
        torch.autograd.graph.increment_version([p for p, _ in items])
        return loss


def reference_param_groups(model, lr):
    """lightning_module.py:185-188: encoder at lr, seg_head at lr*10."""
    return [{"params": list(model.encoder.parameters()), "lr": lr},
            {"params": list(model.seg_head.parameters()), "lr": lr * 10}]
