"""All of a trainer's optimiser steps as ONE kernel launch (tgfr_optim_step).

The reference steps torch.optim.Adam for the heads and torch.optim.SGD for the
ArcMargin classifiers (src/train_encoders_bert.py:212-222, :323-330;
src/fusion_bert.py:119-139, :238-239).  ``FusedOptimizer`` holds both as
parameter groups and updates every tensor in one launch; the update rules are
torch's (include/tgfr.h, 'optimiser step').  The step count is kept on the
device, so a step captured into a HIP graph replays correctly; so are the
per-group learning-rate factors, so ``set_lr`` / ``scale_lr`` (the reference's
ExponentialLR(gamma=0.98) on the head and its 10x classifier cuts,
src/train_encoders_bert.py:225, :406-410) take effect at the next step, also
on a captured step that is replayed without re-capture.

    opt = FusedOptimizer([adam_group(head.parameters(), lr=2e-4, betas=(0.5, 0.999)),
                          sgd_group(cls.parameters(), lr=0.1, momentum=0.9,
                                    weight_decay=5e-5)])
    opt.zero_grad(set_to_none=True); loss.backward(); opt.step()
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _hip

ADAM, SGD = 0, 1
MAX_SEGS, MAX_GROUPS = 48, 4


class _Group(C.Structure):
    _fields_ = [("kind", C.c_int), ("lr", C.c_float), ("beta1", C.c_float),
                ("beta2", C.c_float), ("eps", C.c_float), ("weight_decay", C.c_float),
                ("momentum", C.c_float), ("dampening", C.c_float)]


class _Seg(C.Structure):
    _fields_ = [("param", C.c_void_p), ("grad", C.c_void_p), ("state0", C.c_void_p),
                ("state1", C.c_void_p), ("n", C.c_longlong), ("group", C.c_int),
                ("reserved", C.c_int)]


def adam_group(params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
    return {"kind": ADAM, "params": list(params), "lr": lr, "betas": tuple(betas),
            "eps": eps, "weight_decay": weight_decay}


def sgd_group(params, lr, momentum=0.0, dampening=0.0, weight_decay=0.0):
    return {"kind": SGD, "params": list(params), "lr": lr, "momentum": momentum,
            "dampening": dampening, "weight_decay": weight_decay}


class FusedOptimizer:
    def __init__(self, groups):
        groups = [g for g in groups if g["params"]]
        if not groups or len(groups) > MAX_GROUPS:
            raise ValueError(f"1..{MAX_GROUPS} non-empty parameter groups")
        self.groups = groups
        self.params = [p for g in groups for p in g["params"]]
        if len(self.params) > MAX_SEGS:
            raise ValueError(f"at most {MAX_SEGS} parameter tensors")
        dev = self.params[0].device
        for p in self.params:
            if p.device != dev or p.dtype != torch.float32 or not p.is_contiguous():
                raise ValueError("parameters must be contiguous fp32 tensors on one device")
        self.state = {}
        for g in groups:
            for p in g["params"]:
                st = []
                if g["kind"] == ADAM:
                    st = [torch.zeros_like(p), torch.zeros_like(p)]
                elif g.get("momentum", 0.0) != 0.0:
                    st = [torch.zeros_like(p)]
                self.state[p] = st
        # [steps taken, last-arriver count]
        self.counters = torch.zeros(2, dtype=torch.int32, device=dev)
        # per-group multipliers of the captured base lr, read by the kernel
        self.base_lr = [float(g["lr"]) for g in groups]
        self.lr_scale = torch.ones(len(groups), dtype=torch.float32, device=dev)
        self._groups_c = (_Group * len(groups))()
        for i, g in enumerate(groups):
            c = self._groups_c[i]
            c.kind = g["kind"]
            c.lr = g["lr"]
            c.weight_decay = g["weight_decay"]
            if g["kind"] == ADAM:
                c.beta1, c.beta2 = g["betas"]
                c.eps = g["eps"]
            else:
                c.momentum = g["momentum"]
                c.dampening = g["dampening"]
        self._segs_c = (_Seg * len(self.params))()

    def get_lr(self, group):
        """The learning rate group `group` uses at the next step (host value)."""
        return self.groups[group]["lr"]

    def set_lr(self, group, lr):
        """Set group `group`'s learning rate for the following steps (one tiny
        device write; no re-capture of a graphed step needed)."""
        lr = float(lr)
        self.groups[group]["lr"] = lr
        base = self.base_lr[group]
        with torch.no_grad():
            self.lr_scale[group].fill_(lr / base if base != 0.0 else 0.0)
        if base == 0.0 and lr != 0.0:
            raise ValueError("cannot rescale a group created with lr = 0")

    def scale_lr(self, group, gamma):
        """lr *= gamma for one group (ExponentialLR.step, the 0.1 cuts)."""
        self.set_lr(group, self.groups[group]["lr"] * gamma)

    @property
    def param_groups(self):
        """torch.optim-style view: one dict per group with its current 'lr'."""
        return self.groups

    @property
    def step_count(self):
        return int(self.counters[0].item())

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    @torch.no_grad()
    def step(self):
        """Update every parameter that has a gradient (one launch)."""
        n = 0
        segs = self._segs_c
        for gi, g in enumerate(self.groups):
            for p in g["params"]:
                if p.grad is None:
                    continue
                gr = p.grad
                if gr.dtype != torch.float32 or not gr.is_contiguous():
                    gr = p.grad = gr.float().contiguous()
                st = self.state[p]
                s = segs[n]
                s.param = _hip.ptr(p)
                s.grad = _hip.ptr(gr)
                s.state0 = _hip.ptr(st[0]) if st else None
                s.state1 = _hip.ptr(st[1]) if len(st) > 1 else None
                s.n = p.numel()
                s.group = gi
                n += 1
        if n == 0:
            return
        _hip.call("tgfr_optim_step", C.addressof(segs), n, C.addressof(self._groups_c),
                  len(self.groups), _hip.ptr(self.lr_scale), _hip.ptr(self.counters),
                  _hip.stream())

