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

Every collective goes through ``all_gather_cat`` / ``all_reduce_sum_``.  While
a ``StepCapture`` is recording a step, each of them closes the HIP graph being
captured, runs the collective eagerly on static buffers (and remembers it), and
opens the next graph, so a distributed step replays as
``graph, collective, graph, collective, ..., graph`` with no host work besides
the launches (train.GraphedStep).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

_CAPTURE = None
_SIDE = {}          # per-device side stream of the eager overlapped collectives


def active_capture():
    return _CAPTURE


class StepCapture:
    """A step captured as a chain of HIP graphs cut at its collectives.

    Graphs share one memory pool, so tensors made in one segment stay valid in
    the next; the collectives between them run on buffers allocated during the
    capture (static addresses), replayed in the captured order."""

    def __init__(self):
        self.graphs = []
        self.collectives = []
        self.pool = torch.cuda.graph_pool_handle()
        self.stream = torch.cuda.Stream()
        self.side = torch.cuda.Stream()       # overlapped collectives (cut_async)

    def _begin(self):
        g = torch.cuda.CUDAGraph()
        g.capture_begin(pool=self.pool)
        self.graphs.append(g)

    def cut(self, fn):
        """Close the current graph, run collective `fn` now and at every
        replay between this graph and the next, open the next graph."""
        self.graphs[-1].capture_end()
        fn()
        self.collectives.append(fn)
        self._begin()

    def cut_async(self, fn):
        """Close the current graph; run collective `fn` on the side stream
        (after everything captured so far) now and at every replay, so that
        the next graphs overlap it; returns the event that join() waits on."""
        self.graphs[-1].capture_end()
        ev = torch.cuda.Event()

        def launch():
            cur = torch.cuda.current_stream()
            self.side.wait_stream(cur)
            with torch.cuda.stream(self.side):
                fn()
            ev.record(self.side)
        launch()
        self.collectives.append(launch)
        self._begin()
        return ev

    def join(self, ev):
        """Close the current graph; the next graphs start after `ev` (an
        overlapped collective of cut_async) completes."""
        self.graphs[-1].capture_end()

        def wait():
            torch.cuda.current_stream().wait_event(ev)
        wait()
        self.collectives.append(wait)
        self._begin()

    def capture(self, step, *args):
        """Record `step(*args)` (on a side stream); returns its outputs, whose
        storage the replays rewrite."""
        global _CAPTURE
        from ._hip import counters
        self.stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self.stream):
            counters(torch.cuda.current_device())      # the capture stream's own words
            self._begin()
            _CAPTURE = self
            try:
                out = step(*args)
            finally:
                _CAPTURE = None
                self.graphs[-1].capture_end()
        torch.cuda.current_stream().wait_stream(self.stream)
        return out

    def replay(self):
        for i, g in enumerate(self.graphs):
            g.replay()
            if i < len(self.collectives):
                self.collectives[i]()


class ReplicaGroup:
    """A stand-in process group for ONE process that plays rank 0 of `world`
    identical replicas (bench.py --simulate-world): gathers repeat the local
    tensor, sums multiply it by `world`.  It reproduces the per-GPU work of a
    `world`-GPU step (B_l images against B_l * world captions) on one device;
    it moves no bytes between devices, so it says nothing about collectives."""

    def __init__(self, world):
        self.world = int(world)


class DistContext:
    def __init__(self, group=None):
        if isinstance(group, ReplicaGroup):
            self.group = group
            self.rank, self.world = 0, group.world
        elif dist.is_available() and dist.is_initialized():
            # an explicit handle: None means "not distributed" to the kernels
            self.group = group if group is not None else dist.group.WORLD
            self.rank = dist.get_rank(self.group)
            self.world = dist.get_world_size(self.group)
        else:
            self.group = None
            self.rank, self.world = 0, 1
        self.active = self.world > 1
        self.b_local = None

    @property
    def multiprocess(self):
        """True when other processes take part (a real process group)."""
        return self.active and not isinstance(self.group, ReplicaGroup)

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
            t = t.detach().clone()
            all_reduce_sum_(t, self.group)
        return t

    def gather_text(self, *tensors):
        """All-gather several equally-batched tensors (any dtypes) along dim 0
        with ONE collective: their bytes are packed per rank, gathered, and
        unpacked rank-major."""
        if not self.active:
            return tensors
        flat = [t.contiguous().view(torch.uint8).reshape(t.shape[0], -1) for t in tensors]
        widths = [f.shape[1] for f in flat]
        packed = torch.cat(flat, 1)
        allp = all_gather_cat(packed, self.group)
        outs, c = [], 0
        for t, w in zip(tensors, widths):
            part = allp[:, c:c + w].contiguous().view(t.dtype)
            outs.append(part.reshape((allp.shape[0],) + tuple(t.shape[1:])))
            c += w
        return tuple(outs)

    def gather_text_async(self, *tensors):
        """gather_text started on a side stream after the current stream's
        work (StepCapture.cut_async under capture), so that the work launched
        next -- IMIM's forward in the DP step -- overlaps the all-gather;
        returns finish(), which orders the current stream after the
        collective (a join) and unpacks the gathered tensors.  gloo (CPU
        tests) gathers synchronously."""
        if not self.active:
            return lambda: tensors
        flat = [t.contiguous().view(torch.uint8).reshape(t.shape[0], -1) for t in tensors]
        widths = [f.shape[1] for f in flat]
        packed = torch.cat(flat, 1)
        allp, ev = all_gather_cat_async(packed, self.group)

        def finish():
            _join(ev)
            _ = packed      # alive until the collective is joined (its block must
            outs, c = [], 0  # not be handed to the overlapped work's tensors)
            for t, w in zip(tensors, widths):
                part = allp[:, c:c + w].contiguous().view(t.dtype)
                outs.append(part.reshape((allp.shape[0],) + tuple(t.shape[1:])))
                c += w
            return tuple(outs)
        return finish

    def reduce_grads_async(self, params):
        """reduce_grads of `params` started now and overlapped with the work
        that follows (a side stream; a cut of its own under StepCapture);
        returns a handle for wait_grads.  For gradients that are final early
        in the step (the identity heads' classifiers, after their branch's
        backward) while the word<->region branch still runs."""
        if not self.active:
            return None
        ps = [p for p in params if p.grad is not None]
        if not ps:
            return None
        flat = torch.cat([p.grad.reshape(-1) for p in ps])
        off = 0
        for p in ps:
            n = p.numel()
            p.grad = flat[off:off + n].view_as(p)
            off += n
        return all_reduce_sum_async_(flat, self.group)

    def wait_grads(self, handle):
        """Order the current stream after a reduce_grads_async."""
        if handle is not None:
            _join(handle)

    def reduce_grads(self, params, after=None):
        """Sum the gradients of `params` over ranks in one all-reduce of a flat
        buffer (the DDP replacement: losses are pre-weighted so that the SUM is
        the global-batch gradient); p.grad become views of the reduced buffer.
        after: a reduce_grads_async handle the current stream also waits for
        here (one step boundary for both buckets under StepCapture)."""
        if not self.active:
            _join(after)
            return
        ps = [p for p in params if p.grad is not None]
        if not ps:
            _join(after)
            return
        flat = torch.cat([p.grad.reshape(-1) for p in ps])
        all_reduce_sum_(flat, self.group, after=after)
        off = 0
        for p in ps:
            n = p.numel()
            p.grad = flat[off:off + n].view_as(p)
            off += n

    def broadcast_params(self, params):
        """Rank 0's initial parameters to every rank (DDP's construction-time
        broadcast)."""
        if not self.active:
            return
        if isinstance(self.group, ReplicaGroup):
            return
        with torch.no_grad():
            for p in params:
                if dist.get_backend(self.group) == "gloo" and p.is_cuda:
                    c = p.detach().cpu()
                    dist.broadcast(c, 0, group=self.group)
                    p.copy_(c)
                else:
                    dist.broadcast(p.data, 0, group=self.group)


def _run_or_cut(fn):
    if _CAPTURE is not None:
        _CAPTURE.cut(fn)
    else:
        fn()


def all_gather_cat(t, group=None):
    """all_gather + concatenate along dim 0 into a fresh tensor.  RCCL gathers
    device tensors in place; gloo (CPU tests) only gathers host tensors, so it
    stages through host memory.  Capture-aware (StepCapture)."""
    t = t.contiguous()
    replica = isinstance(group, ReplicaGroup)
    world = group.world if replica else dist.get_world_size(group)
    out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype,
                      device=t.device)
    gloo = not replica and dist.get_backend(group) == "gloo"

    def run():
        if replica:
            out.view((world,) + tuple(t.shape)).copy_(t.unsqueeze(0).expand(
                (world,) + tuple(t.shape)))
        elif gloo:
            src = t.cpu() if t.is_cuda else t
            parts = [torch.empty_like(src) for _ in range(world)]
            dist.all_gather(parts, src, group=group)
            out.copy_(torch.cat(parts, 0))
        else:
            dist.all_gather_into_tensor(out, t, group=group)
    _run_or_cut(run)
    return out


def all_gather_cat_async(t, group=None):
    """all_gather_cat started on a side stream after the current stream's work
    (StepCapture.cut_async under capture): returns (out, event to join before
    reading out).  gloo (CPU tests): synchronous, event None."""
    t = t.contiguous()
    replica = isinstance(group, ReplicaGroup)
    if not replica and dist.get_backend(group) == "gloo":
        return all_gather_cat(t, group), None
    world = group.world if replica else dist.get_world_size(group)
    out = torch.empty((world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype,
                      device=t.device)

    def run():
        if replica:
            out.view((world,) + tuple(t.shape)).copy_(t.unsqueeze(0).expand(
                (world,) + tuple(t.shape)))
        else:
            dist.all_gather_into_tensor(out, t, group=group)
    if _CAPTURE is not None:
        return out, _CAPTURE.cut_async(run)
    dev = torch.cuda.current_device()
    side = _SIDE.setdefault(dev, torch.cuda.Stream())
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        run()
    ev = torch.cuda.Event()
    ev.record(side)
    t.record_stream(side)
    out.record_stream(side)
    return out, ev


def all_reduce_sum_(t, group=None, after=None):
    """In-place SUM all-reduce (gloo stages device tensors through host
    memory).  Capture-aware (StepCapture).  after: an event (of an overlapped
    collective) the current stream waits for first -- inside the same step
    boundary under capture."""
    replica = isinstance(group, ReplicaGroup)
    gloo = not replica and dist.get_backend(group) == "gloo"

    def run():
        if after is not None:
            torch.cuda.current_stream().wait_event(after)
        if replica:
            t.mul_(group.world)
        elif gloo and t.is_cuda:
            c = t.cpu()
            dist.all_reduce(c, group=group)
            t.copy_(c)
        else:
            dist.all_reduce(t, group=group)
    _run_or_cut(run)
    return t


def all_reduce_sum_async_(t, group=None):
    """In-place SUM all-reduce started on a side stream after the current
    stream's work (capture-aware: StepCapture.cut_async); returns the event
    to join.  gloo (CPU tests) stages through host memory synchronously."""
    replica = isinstance(group, ReplicaGroup)
    if not replica and dist.get_backend(group) == "gloo":
        all_reduce_sum_(t, group)
        return None

    def run():
        if replica:
            t.mul_(group.world)
        else:
            dist.all_reduce(t, group=group)
    if _CAPTURE is not None:
        return _CAPTURE.cut_async(run)
    dev = torch.cuda.current_device()
    side = _SIDE.setdefault(dev, torch.cuda.Stream())
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        run()
    ev = torch.cuda.Event()
    ev.record(side)
    t.record_stream(side)
    return ev


def _join(ev):
    if ev is None:
        return
    if _CAPTURE is not None:
        _CAPTURE.join(ev)
    else:
        torch.cuda.current_stream().wait_event(ev)


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
