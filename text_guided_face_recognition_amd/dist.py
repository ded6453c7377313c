"""Data parallelism: one process per GPU, torch.distributed over RCCL/xGMI.

The reference runs nn.DataParallel (single process, losses on GPU 0 over the
gathered batch; src/train_encoders_bert.py:146-169).  Here every rank keeps
its own images and gathers only what the contrastive denominators need:

  * all_gather of the text side (words W, sentence vectors, class ids) --
    detached in the reference (utils/dataset_utils.py:42), so no backward
    collective is needed for it;
  * one all_gather of the per-column (max, sum-exp) partials inside
    kernels.ContrastiveCE so loss1 sees every rank's images;
  * the DDP gradient all-reduce of the trainable heads.

Rank r owns global rows [r*B_l, (r+1)*B_l) (rank-major), the same order the
reference's gathered batch has, so the summed per-rank losses equal the
single-process global-batch losses.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


class DistContext:
    def __init__(self, group=None):
        if dist.is_available() and dist.is_initialized():
            # an explicit handle: None means "not distributed" to the kernels
            self.group = group if group is not None else dist.group.WORLD
            self.rank = dist.get_rank(self.group)
            self.world = dist.get_world_size(self.group)
        else:
            self.group = None
            self.rank, self.world = 0, 1
        self.active = self.world > 1
        self.b_local = None

    def set_batch(self, b_local):
        self.b_local = int(b_local)
        return self

    @property
    def row_offset(self):
        return self.rank * self.b_local

    @property
    def n_global(self):
        return self.world * self.b_local

    def gather_rows(self, t):
        """Concatenate equally-shaped per-rank tensors along dim 0 (rank-major)."""
        if not self.active:
            return t
        return all_gather_cat(t, self.group)

    def sum(self, t):
        if self.active:
            if dist.get_backend(self.group) == "gloo" and t.is_cuda:
                c = t.detach().cpu()
                dist.all_reduce(c, group=self.group)
                return c.to(t.device)
            t = t.clone()
            dist.all_reduce(t, group=self.group)
        return t


def all_gather_cat(t, group=None):
    """all_gather + concatenate along dim 0.  RCCL gathers device tensors in
    place; gloo (CPU tests) only gathers host tensors, so it stages through host
    memory."""
    t = t.contiguous()
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "gloo" and t.is_cuda:
        parts = [torch.empty_like(t, device="cpu") for _ in range(world)]
        dist.all_gather(parts, t.cpu(), group=group)
        return torch.cat(parts, 0).to(t.device)
    if dist.get_backend(group) == "gloo":
        parts = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(parts, t, group=group)
        return torch.cat(parts, 0)
    out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype,
                      device=t.device)
    dist.all_gather_into_tensor(out, t, group=group)
    return out


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's env (127.0.0.1)."""
    if "WORLD_SIZE" not in os.environ or int(os.environ["WORLD_SIZE"]) <= 1:
        return DistContext()
    if not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("TGFR_DIST_BACKEND") or (
                "nccl" if torch.cuda.device_count() > 0 else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
        dist.init_process_group(backend=backend)
    return DistContext()
