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


class _GroupView(dict):
    """One entry of ``FusedOptimizer.param_groups``: a torch.optim-style dict
    whose ``g['lr'] = x`` goes through ``set_lr`` (the reference cuts the
    classifier lr that way, src/train_encoders_bert.py:408-410), so the kernel
    applies exactly the lr the dict reports."""

    def __init__(self, opt, index, group):
        super().__init__(group)
        self._opt, self._index = opt, index

    def __setitem__(self, key, value):
        if key == "lr":
            self._opt.set_lr(self._index, value)      # validates, then mirrors here
            return
        if key in self and self[key] != value:
            raise ValueError(f"param group key {key!r} is fixed at construction "
                             "(only 'lr' can change between steps)")
        super().__setitem__(key, value)


class FusedOptimizer:
    def __init__(self, groups):
        groups = list(groups)
        # caller's group index -> internal index (None for an empty group, which
        # keeps its slot so set_lr / scale_lr / param_groups indices match the
        # caller's list, as in torch.optim)
        self._index = []
        kept = []
        for g in groups:
            self._index.append(len(kept) if g["params"] else None)
            if g["params"]:
                kept.append(g)
        if not kept or len(kept) > MAX_GROUPS:
            raise ValueError(f"1..{MAX_GROUPS} non-empty parameter groups")
        self._all_groups = groups
        groups = kept
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
        """The learning rate group `group` (caller's index) uses at the next
        step (host value)."""
        return float(self._all_groups[group]["lr"])

    def set_lr(self, group, lr):
        """Set group `group`'s learning rate (caller's index) for the following
        steps (one tiny device write; no re-capture of a graphed step needed).
        Validated before anything changes."""
        lr = float(lr)
        gi = self._index[group]
        if gi is not None:
            base = self.base_lr[gi]
            if base == 0.0 and lr != 0.0:
                raise ValueError("cannot rescale a group created with lr = 0")
            with torch.no_grad():
                self.lr_scale[gi].fill_(lr / base if base != 0.0 else 0.0)
        self._all_groups[group]["lr"] = lr
        views = self.__dict__.get("_views")
        if views is not None:
            dict.__setitem__(views[group], "lr", lr)

    def scale_lr(self, group, gamma):
        """lr *= gamma for one group (ExponentialLR.step, the 0.1 cuts)."""
        self.set_lr(group, self.get_lr(group) * gamma)

    @property
    def param_groups(self):
        """torch.optim-style view: one dict per group (the caller's order, empty
        groups included) with its current 'lr'; ``g['lr'] = x`` is applied to
        the next step exactly like ``set_lr``."""
        views = self.__dict__.get("_views")
        if views is None:
            views = self._views = [_GroupView(self, i, g)
                                   for i, g in enumerate(self._all_groups)]
        return views

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
    def step(self, groups=None):
        """Update every parameter that has a gradient (one launch).  groups: a
        subset of the caller's group indices to update in this launch (the
        rest wait for another call); a subset without an Adam group does not
        advance the step count (its launch counts on a private counter, so
        two subset launches may run concurrently on two streams)."""
        n = 0
        segs = self._segs_c if groups is None else (_Seg * len(self.params))()
        only = None if groups is None else {self._index[i] for i in groups} - {None}
        for gi, g in enumerate(self.groups):
            if only is not None and gi not in only:
                continue
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
        counters = self.counters
        aux = only is not None and all(self.groups[gi]["kind"] != ADAM for gi in only)
        if aux:
            counters = self.__dict__.get("_aux_counters")
            if counters is None:
                counters = self._aux_counters = torch.zeros_like(self.counters)
        # a group's first-step flag (SGD momentum init) comes from the counter
        # its launch counts on: one group must always count on the same one
        # (calling it through an Adam-free subset and through a full step()
        # would re-initialise its momentum, or never initialise it)
        which = self.__dict__.setdefault("_counter_of", {})
        for gi in (range(len(self.groups)) if only is None else only):
            prev = which.setdefault(gi, aux)
            if prev != aux:
                raise RuntimeError(
                    f"optimiser group {gi} was stepped both through an Adam-free subset "
                    "step(groups=...) and through a step that advances the main counter; "
                    "use one calling mode per group")
        _hip.call("tgfr_optim_step", C.addressof(segs), n, C.addressof(self._groups_c),
                  len(self.groups), _hip.ptr(self.lr_scale), _hip.ptr(counters),
                  _hip.stream())

