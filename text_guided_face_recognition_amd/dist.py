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
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.world = dist.get_world_size(group)
        else:
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
        t = t.contiguous()
        out = torch.empty((self.world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype,
                          device=t.device)
        dist.all_gather_into_tensor(out, t, group=self.group)
        return out

    def sum(self, t):
        if self.active:
            t = t.clone()
            dist.all_reduce(t, group=self.group)
        return t


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's env (127.0.0.1)."""
    if "WORLD_SIZE" not in os.environ or int(os.environ["WORLD_SIZE"]) <= 1:
        return DistContext()
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
        dist.init_process_group(backend=backend)
    return DistContext()
