"""CPU, world_size 2 over gloo: the rank-major row ownership, the text-side
all-gather (one packed collective for mixed dtypes), the column log-sum-exp
exchange of the contrastive CE, the flat gradient all-reduce and the initial
parameter broadcast reproduce the single-process global-batch quantities."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from text_guided_face_recognition_amd.dist import DistContext
        from text_guided_face_recognition_amd.kernels import gather_col_partials

        def combine_col_partials(parts):
            # the math of tgfr_col_lse_combine.  The shipped combine is that
            # kernel alone (no CPU fallback by design, tests/test_abi.py
            # ::test_device_only_contract), so this CPU test covers the
            # exchange layout and the collective; the kernel itself is checked
            # on the GPU against this same math (tests/test_gpu_dp.py
            # ::test_dp_glue_kernels)
            gmax = parts[:, 0].max(0).values
            return gmax + torch.log((parts[:, 1] * torch.exp(parts[:, 0] - gmax)).sum(0))

        def exchange_col_partials(part, group):
            return combine_col_partials(gather_col_partials(part, group))
        torch.manual_seed(0)
        b_l = 3
        full = torch.randn(world * b_l, world * b_l) * 4            # global logits
        text = torch.randn(world * b_l, 5)
        ctx = DistContext().set_batch(b_l)
        mine = full[ctx.row_offset:ctx.row_offset + b_l]
        # text side: each rank holds its own rows and gathers the global batch
        gathered = ctx.gather_rows(text[ctx.row_offset:ctx.row_offset + b_l])
        ok_gather = torch.equal(gathered, text)
        # column partials of this rank's row block, as tgfr_ce_stats computes them
        cmax = mine.max(0).values
        part = torch.stack([cmax, torch.exp(mine - cmax).sum(0)])
        col_lse = exchange_col_partials(part, ctx.group)
        ok_lse = torch.allclose(col_lse, torch.logsumexp(full, 0), atol=1e-5)
        # per-rank CE contributions sum to the global losses
        n = world * b_l
        idx = torch.arange(ctx.row_offset, ctx.row_offset + b_l)
        diag = mine[torch.arange(b_l), idx]
        l0 = (torch.logsumexp(mine, 1) - diag).sum() / n
        l1 = (col_lse[idx] - diag).sum() / n
        tot = ctx.sum(torch.stack([l0, l1]))
        lab = torch.arange(n)
        ref = torch.stack([torch.nn.functional.cross_entropy(full, lab),
                           torch.nn.functional.cross_entropy(full.t(), lab)])
        ok_loss = torch.allclose(tot, ref, atol=1e-5)
        one = combine_col_partials(part.unsqueeze(0))
        ok_single = torch.allclose(one, torch.logsumexp(mine, 0), atol=1e-5)
        # packed text gather: fp32 words [B, T, D], fp32 sentences, int64 ids
        words = torch.randn(world * b_l, 4, 6)
        sent = torch.randn(world * b_l, 6)
        ids = torch.randint(0, 10 ** 12, (world * b_l,))
        rows = slice(ctx.row_offset, ctx.row_offset + b_l)
        gw, gs, gi = ctx.gather_text(words[rows].transpose(1, 2), sent[rows], ids[rows])
        ok_gather = ok_gather and torch.equal(gw, words.transpose(1, 2)) and \
            torch.equal(gs, sent) and torch.equal(gi, ids) and gi.dtype == torch.int64
        # broadcast of rank 0's parameters, then the summed flat gradient
        torch.manual_seed(1 + rank)                     # different init per rank
        lin = torch.nn.Linear(6, 3)
        ctx.broadcast_params(list(lin.parameters()))
        torch.manual_seed(1)
        ref_lin = torch.nn.Linear(6, 3)
        ok_bcast = all(torch.equal(a, b) for a, b in zip(lin.parameters(),
                                                         ref_lin.parameters()))
        x = torch.randn(world * b_l, 6)
        lin(x[rows]).pow(2).sum().backward()
        ctx.reduce_grads(list(lin.parameters()))
        ref_lin(x).pow(2).sum().backward()
        ok_grad = all(torch.allclose(a.grad, b.grad, atol=1e-5)
                      for a, b in zip(lin.parameters(), ref_lin.parameters()))
        ok_gather = ok_gather and ok_bcast and ok_grad
        q.put((rank, ok_gather, ok_lse, ok_loss, ok_single, ctx.n_global))
    finally:
        dist.destroy_process_group()


def test_dp_exchange_world2():
    world = 2
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_gather, ok_lse, ok_loss, ok_single, n_global in res:
        assert ok_gather and ok_lse and ok_loss and ok_single, (rank, res)
        assert n_global == 6
