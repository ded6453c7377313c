"""Train-step mirrors of the reference trainers, on frozen-encoder features.

  Train   src/train_encoders_bert.py:233-331 (stage 1, FCAM): image head (IMIM)
          -> words_loss + sent_loss (DAMSM) + 2 ArcMargin/focal identity
          losses + global_loss (CLIP term) -> backward -> optimiser steps.
  TrainLSTM  src/train_encoders_lstm.py:236-314 (stage 1, LSTM text encoder,
          BASELINE configs[0]): words_loss with per-caption lengths (w0 + w1;
          the reference computes sent_loss and discards it, :263-266) +
          2 ArcMargin/focal identity losses + lambda_clip * ClipLoss (:288-291).
  Fusion  src/fusion_bert.py:195-243 (stage 2, FCFM): image head -> Working
          -> ArcMargin(640) -> focal loss -> backward -> optimiser steps.

The frozen encoders of the reference (iResNet, BERT + TextHeading under
no_grad, utils/dataset_utils.py:38-46) are outside the hot path: a step takes
their outputs (global [B,512], layer3 map [B,256,14,14], words [B,256,T],
sentence [B,256], class ids) as device tensors.  ``synthetic_batch`` makes
them with the shapes and statistics SURVEY.md 8(d) prescribes.

One process per GPU: pass a DistContext; text features and class ids are
all-gathered (one collective) so every contrastive denominator sees the global
batch.  Gradients are summed over ranks by one flat all-reduce
(DistContext.reduce_grads, in place of DDP).  The contrastive losses are this
rank's contributions to the global-batch losses; the focal identity losses are
formed from the GLOBAL mean cross-entropy (one all-reduce of the per-rank NLL
sums, kernels.FocalCE), as the reference's DataParallel computes them on the
gathered batch.  Every term enters with the reference's weight, and the
summed gradient is the reference's global-batch gradient.  Initial parameters
are broadcast from rank 0.
"""
from __future__ import annotations

import os

import torch
from . import kernels as K
from .dist import DistContext, StepCapture
from .models.fusion_nets import Working, set_precision
from .models.losses import (ClipLoss, FocalLoss, _class_tensor, sent_global_loss, words_loss,
                            words_logits_bert)
from .models.metrics import ArcMarginProduct
from .models.models import ImageHeading, TextHeading
from .optim import FusedOptimizer, adam_group, sgd_group


def _unit(x, dim=-1):
    return x / x.norm(dim=dim, keepdim=True)


def synthetic_batch(b, n_words, device, seed, n_ids=10000, bert_hidden=False):
    """Frozen-encoder outputs for one batch: (global, local,
    words [B, 256, T], sent, class ids), or with bert_hidden the BERT-base
    last hidden states without [CLS] instead of the text features -- (global,
    local, hidden [B, T + 1, 768], class ids) -- so that the step runs the
    frozen TextHeading itself, as the reference's does
    (utils/dataset_utils.py:38-46)."""
    gen = torch.Generator(device="cpu").manual_seed(seed)
    g = torch.randn(b, 512, generator=gen)
    local = torch.randn(b, 256, 14, 14, generator=gen)
    to = dict(device=device)
    if bert_hidden:
        hidden = torch.randn(b, n_words + 1, 768, generator=gen)
        cls = torch.randint(0, n_ids, (b,), generator=gen)
        return g.to(**to), local.to(**to), hidden.to(**to), cls.to(**to)
    words = _unit(torch.randn(b, n_words, 256, generator=gen))     # [B, T, 256] storage
    sent = _unit(torch.randn(b, 256, generator=gen))
    cls = torch.randint(0, n_ids, (b,), generator=gen)
    return (g.to(**to), local.to(**to), words.to(**to).transpose(1, 2), sent.to(**to),
            cls.to(**to))


def synthetic_batch_lstm(b, max_words, device, seed, n_ids=1000):
    """Frozen BiLSTM-encoder outputs for one batch:
    words [B, 256, Lmax] (unnormalised, tanh-range like the LSTM's outputs,
    models/models.py:311-318; storage [B, Lmax, 256]), sentence codes
    L2-normalised (:323), caption lengths U[3, Lmax] (device int32)."""
    gen = torch.Generator(device="cpu").manual_seed(seed)
    g = torch.randn(b, 512, generator=gen)
    local = torch.randn(b, 256, 14, 14, generator=gen)
    words = torch.tanh(torch.randn(b, max_words, 256, generator=gen))
    sent = _unit(torch.randn(b, 256, generator=gen))
    cls = torch.randint(0, n_ids, (b,), generator=gen)
    lens = torch.randint(3, max_words + 1, (b,), generator=gen)
    to = dict(device=device)
    return (g.to(**to), local.to(**to), words.to(**to).transpose(1, 2), sent.to(**to),
            cls.to(**to), lens.to(device=device, dtype=torch.int32))


class Train:
    """Stage-1 BERT trainer step (src/train_encoders_bert.py)."""

    _forks = True       # step() takes _step_forked on one process (subclasses may not)

    def __init__(self, args, device, ctx=None):
        self.args = args
        self.ctx = ctx or DistContext()
        args.return_att_maps = False
        self.image_head = ImageHeading(args).to(device)
        self.image_cls = ArcMarginProduct(args.aux_feat_dim_per_granularity,
                                          args.num_classes, s=30, m=0.5).to(device)
        # the frozen text head (:212 puts its parameters in the Adam group, but
        # it runs under no_grad, utils/dataset_utils.py:42-45, so they never
        # change); used when a batch carries BERT hidden states
        self.text_head = TextHeading(args).to(device).requires_grad_(False)
        set_precision(self.text_head, args.precision)
        self.text_cls = ArcMarginProduct(args.aux_feat_dim_per_granularity,
                                         args.num_classes, s=35, m=0.5).to(device)
        for m in (self.image_head, self.image_cls, self.text_cls):
            set_precision(m, args.precision)
        self.head_params = list(self.image_head.parameters())
        self.cls_params = list(self.image_cls.parameters()) + list(self.text_cls.parameters())
        self.params = self.head_params + self.cls_params
        # the frozen text head too: every rank must make its captions with the
        # same weights, or the gathered words mix different text heads
        self.ctx.broadcast_params(self.params + list(self.text_head.parameters()))
        self.ident_loss = FocalLoss(gamma=2)
        # one process: the g' branch (projection head, sentence / global
        # losses, both identity heads, their backward) runs on a side stream
        # beside IMIM and the word<->region branch -- its kernels are small
        # latency chains that leave most of the chip idle
        # (TGFR_FORK: 0 = one linear stream, 1 = the g' branch forked, 2 = the
        # frozen TextHeading heading that side stream too; round 4 at config 2:
        # 0.547 / 0.482 / 0.460 ms per step; the classifiers' SGD step on the
        # side stream as well, _step_forked.  The logged-loss mix there costs
        # a cross-stream edge and measured slower: 0.50 ms)
        # With a process group the forked step is _step_forked_dp (its three
        # mid-step collectives merged into one, so the fork is not cut apart).
        fork = os.environ.get("TGFR_FORK", "2")
        self.fork = self._forks and fork != "0"
        self.fork_text = fork == "2"
        self._side = torch.cuda.Stream(device) if self.fork and torch.cuda.is_available() else None
        # :212 (text_head params would join here; the text side is frozen input)
        # :212 Adam for the head, :219-222 SGD for both classifiers: one launch
        self.optimizer = FusedOptimizer([
            adam_group(self.image_head.parameters(), lr=args.lr_head, betas=(0.5, 0.999)),
            sgd_group(list(self.image_cls.parameters()) + list(self.text_cls.parameters()),
                      lr=0.1, momentum=0.9, weight_decay=5e-5)])

    def step(self, batch):
        """batch: (global, local, words, sent, class ids), or (global, local,
        BERT hidden states, class ids) -- then the step runs TextHeading under
        no_grad first (:257, utils/dataset_utils.py:38-46)."""
        if self._side is not None:
            if not self.ctx.active:
                return self._step_forked(batch)
            if self._dp_forkable(batch):
                return self._step_forked_dp(batch)
        args, ctx = self.args, self.ctx
        if len(batch) == 4:
            g, local, hidden, class_ids = batch
            with torch.no_grad():
                words, sent = self.text_head(hidden, None)
        else:
            g, local, words, sent, class_ids = batch
        b = g.shape[0]
        ctx.set_batch(b)
        args.dist = ctx
        # text side: all-gathered global batch (detached, as in the reference)
        words_g, sent_g, cls_g = self._gather_text(words, sent, class_ids)
        labels = self._labels(ctx.n_global, g.device)

        self.optimizer.zero_grad(set_to_none=True)
        wi, lc = float(args.lambda_id), float(args.lambda_clip)
        img_features, words_features = self.image_head(g, local)   # :265

        # total = damsm + lambda_clip * cl + lambda_id * (tid + iid) (:279,
        # :316-323) is linear in the terms, so each term's gradient is its
        # constant weight: every branch runs its backward right after its own
        # forward (no loss-mix backward launch).  With a process group the
        # step stays one linear stream (its collectives cut the graphs).
        s0, s1, cl = sent_global_loss(img_features, sent_g, labels, cls_g, b, args)  # :276, :310
        # :293-306, both focal losses from the global-batch mean CE
        tid, iid = self._identity(sent, img_features, class_ids, ctx)
        torch.autograd.backward((s0, s1, cl, tid, iid),
                                self._weights((1.0, 1.0, lc, wi, wi), g.device))
        # the classifiers' gradients are final here: their all-reduce (9.2 MB
        # at 4500 classes) overlaps the word<->region branch
        pending = ctx.reduce_grads_async(self.cls_params)
        w0, w1, _ = words_loss(words_features, words_g, labels, None, cls_g, b, args)
        torch.autograd.backward((w0, w1), self._weights((1.0, 1.0), g.device))
        return self._finish(w0, w1, s0, s1, cl, tid, iid, lc, wi, pending)

    def _step_forked(self, batch):
        """One process: the reference's :265 forward split over two streams.
        IMIM and the word<->region branch on the current (main) stream; the
        frozen TextHeading (TGFR_FORK=2) and the g' branch (projection head,
        sentence / global losses, identity heads, their backward) on the side
        stream, forked at the step's start; the word<->region branch waits for
        TextHeading's event, the optimiser for the whole side branch.

        Launch order matters under a replayed graph: its nodes are dispatched
        in capture order, so IMIM's forward is launched first (the main
        branch is the critical path).  Round 4 at config 2, three interleaved
        rounds on one box: IMIM first 0.433-0.436 ms per step, the side
        branch first 0.449-0.460, the g' branch after the word<->region
        backward 0.442-0.449, between the word<->region forward and backward
        0.444-0.453 (against 0.433-0.446) (profiles/r04/fork_ab.txt)."""
        args, ctx = self.args, self.ctx
        main, side = torch.cuda.current_stream(), self._side
        start = torch.cuda.Event()
        start.record(main)
        words_features = self.image_head.imim(batch[1])
        side.wait_event(start)
        text_ev = None
        if len(batch) == 4:
            g, local, hidden, class_ids = batch
            if self.fork_text:
                with torch.cuda.stream(side), torch.no_grad():
                    words, sent = self.text_head(hidden, None)
                text_ev = torch.cuda.Event()
                text_ev.record(side)
            else:
                with torch.no_grad():
                    words, sent = self.text_head(hidden, None)
                side.wait_stream(main)       # (after IMIM's forward too)
        else:
            g, local, words, sent, class_ids = batch
        b = g.shape[0]
        ctx.set_batch(b)
        args.dist = ctx
        words_g, sent_g, cls_g = self._gather_text(words, sent, class_ids)
        labels = self._labels(ctx.n_global, g.device)
        self.optimizer.zero_grad(set_to_none=True)
        wi, lc = float(args.lambda_id), float(args.lambda_clip)
        order = os.environ.get("TGFR_ORDER", "a")

        def side_fwd():
            with torch.cuda.stream(side):
                img_features = self.image_head.global_features(g)
                s0, s1, cl = sent_global_loss(img_features, sent_g, labels, cls_g, b, args)
                tid, iid = self._identity(sent, img_features, class_ids, ctx)
            return s0, s1, cl, tid, iid

        def side_bwd(terms):
            with torch.cuda.stream(side):
                torch.autograd.backward(terms, self._weights((1.0, 1.0, lc, wi, wi), g.device))
                # the classifiers' gradients are final: their SGD update (group 1,
                # most of the optimiser's bytes) runs here, beside the
                # word<->region branch (0.434-0.437 -> 0.429-0.430 ms per step)
                self.optimizer.step(groups=[1])

        def wr_fwd():
            if text_ev is not None:
                main.wait_event(text_ev)
            return words_loss(words_features, words_g, labels, None, cls_g, b, args)[:2]

        if order == "a":
            terms = side_fwd()
            side_bwd(terms)
            w0, w1 = wr_fwd()
        elif order == "b":
            terms = side_fwd()
            w0, w1 = wr_fwd()
            side_bwd(terms)
        else:
            w0, w1 = wr_fwd()
            terms = side_fwd()
            side_bwd(terms)
        s0, s1, cl, tid, iid = terms
        torch.autograd.backward((w0, w1), self._weights((1.0, 1.0), g.device))
        main.wait_stream(side)
        return self._finish(w0, w1, s0, s1, cl, tid, iid, lc, wi, None, groups=[0])

    def _dp_forkable(self, batch):
        """The data-parallel forked step needs the fused loss paths: the BERT
        word<->region path without attention maps, this rank's <= 128 images
        (sentence / global and identity-head kernels; configs[4]'s 128 per rank
        included) against <= 8192 gathered captions, and two identity heads of
        one (D, C) and margin."""
        tc, ic = self.text_cls, self.image_cls
        b = batch[0].shape[0]
        return (self.args.en_type == "BERT" and b <= 128 and b * self.ctx.world <= 8192
                and tc.weight.shape == ic.weight.shape and tc.m == ic.m
                and tc.easy_margin == ic.easy_margin)

    def _step_forked_dp(self, batch):
        """One process per GPU: the forked step of _step_forked with the
        reference's DataParallel global-batch semantics
        (src/train_encoders_bert.py:146-169), cut at three collectives:

          1. the text side's all-gather (after the frozen TextHeading, with
             the g' projection beside it);
          2. ONE all-gather of every rank's mid-step partials -- the word<->
             region CE's column (max, sum exp) partials, the sentence / global
             losses' column partials and both identity heads' NLL sums -- packed
             in one buffer by the three losses' first stages (kernels.ce_partials,
             sent_global_dist_parts, identity_heads_parts); their second stages
             read the gathered rows in place (any row stride);
          3. one flat all-reduce of every trained gradient, then ONE optimiser
             launch.  (Splitting it -- the classifiers' bucket on a side stream
             beside IMIM's backward -- cuts the backward into two graphs, and
             the g' branch's backward chain, ~150 us beside the word<->region
             backward alone, then bounds the first: +0.12 ms per rank step in
             the simulate-world-8 configs[2] step, more than the bucket's
             all-reduce it would hide.)

        The g' projection runs beside TextHeading; after 1, IMIM's forward
        beside both identity heads' forwards on the side stream (they need
        only this rank's rows), then the word<->region forward beside the
        sentence / global partials; between 2 and 3 the main stream runs the word<->region
        and IMIM backward while the side runs the g' branch's losses and
        backward.  (Round 5 ran TextHeading, the text gather and IMIM in
        series; the linear DP step cuts at six collectives and a join and runs
        the g' branch in series.)"""
        args, ctx = self.args, self.ctx
        main, side = torch.cuda.current_stream(), self._side
        g = batch[0]
        b = g.shape[0]
        ctx.set_batch(b)
        args.dist = ctx
        dev = g.device
        self.optimizer.zero_grad(set_to_none=True)
        # the g' projection needs only this rank's rows: beside TextHeading
        side.wait_stream(main)
        with torch.cuda.stream(side):
            img_features = self.image_head.global_features(g)
        if len(batch) == 4:
            g, local, hidden, class_ids = batch
            with torch.no_grad():
                words, sent = self.text_head(hidden, None)
        else:
            g, local, words, sent, class_ids = batch
        main.wait_stream(side)
        # (TGFR_TEXT_ASYNC=1: the gather on a side stream beside IMIM's
        # forward -- its join is one more graph boundary, which cost more than
        # a 7 MB gather takes: simulate-world-8 configs[2] 1.290-1.312 against
        # 1.257-1.267 ms per rank step, three interleaved rounds)
        if os.environ.get("TGFR_TEXT_ASYNC", "0") == "1":
            finish_text = self._gather_text_async(words, sent, class_ids)        # 1
        else:
            text_g = self._gather_text(words, sent, class_ids)

            def finish_text():
                return text_g
        wi, lc = float(args.lambda_id), float(args.lambda_clip)
        gamma3, eps, temp3 = args.TRAIN.SMOOTH.GAMMA3, 1e-8, 10.0
        row_offset, n_global = ctx.row_offset, ctx.n_global
        n_c = b * ctx.world
        # this rank's mid-step partials: [words CE 2 n_c | sent/global | NLL sums 2]
        n_sg = K.sent_global_dist_cols(b, n_c)
        buf = torch.empty(2 * n_c + n_sg + 2, dtype=torch.float32, device=dev)
        side.wait_stream(main)
        words_features = self.image_head.imim(local)
        with torch.cuda.stream(side):
            ih = K.identity_heads_parts(sent, self.text_cls, img_features, self.image_cls,
                                        class_ids, self.ident_loss.gamma, buf[2 * n_c + n_sg:])
        main.wait_stream(side)
        words_g, sent_g, cls_g = finish_text()
        assert words_g.shape[0] == n_c
        cls_t = _class_tensor(cls_g, dev)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            sg = K.sent_global_dist_parts(img_features, sent_g, cls_t, gamma3, temp3, eps,
                                          row_offset, buf[2 * n_c:2 * n_c + n_sg])
        logits = words_logits_bert(words_features, words_g, args)
        row_lse = K.ce_partials(logits, buf[:2 * n_c].view(2, n_c))
        main.wait_stream(side)
        from .dist import all_gather_cat
        allp = all_gather_cat(buf.unsqueeze(0), ctx.group)                        # 2
        world = allp.shape[0]
        side.wait_stream(main)
        with torch.cuda.stream(side):
            s0, s1, cl = K.sent_global_dist(img_features, sent_g, cls_t, gamma3, temp3, eps,
                                            row_offset, n_global, ctx.group,
                                            pre=sg + (allp[:, 2 * n_c:2 * n_c + n_sg],))
            tid, iid = K.identity_heads(sent, self.text_cls, img_features, self.image_cls,
                                        class_ids, self.ident_loss.gamma, group=ctx.group,
                                        n_global=n_global,
                                        pre=(ih, allp[:, 2 * n_c + n_sg:]))
            torch.autograd.backward((s0, s1, cl, tid, iid),
                                    self._weights((1.0, 1.0, lc, wi, wi), dev))
        w0, w1 = K.contrastive_ce(logits, row_offset, n_global, ctx.group,
                                  pre=(row_lse, allp[:, :2 * n_c].reshape(world, 2, n_c)))
        torch.autograd.backward((w0, w1), self._weights((1.0, 1.0), dev))
        main.wait_stream(side)
        out = self._report(w0, w1, s0, s1, cl, tid, iid, lc, wi)
        ctx.reduce_grads(self.params)                                             # 3
        self.optimizer.step()
        return out

    def _gather_text_async(self, words, sent, class_ids):
        """_gather_text as gather_text_async: returns finish() -> (words,
        sent, class ids) of the global batch."""
        ctx = self.ctx
        words_bt = words.transpose(1, 2)
        f16 = self.args.precision == "fp16"
        pre = K.attached_rows(words_bt, f16, scale=K.LOG2E) \
            if K.wr_rows_path(self.args.precision, words.shape[2],
                              self.args.en_type == "BERT") else None
        n_words = words.shape[2]
        if pre is not None:
            rows, norms = pre
            fin = ctx.gather_text_async(rows, norms, sent, class_ids)

            def finish():
                rows_g, norms_g, sent_g, cls_g = fin()
                return K.rows_only_words(rows_g, norms_g, n_words, f16), sent_g, cls_g
            return finish
        fin = ctx.gather_text_async(words_bt, sent, class_ids)

        def finish():
            words_g, sent_g, cls_g = fin()
            return words_g.transpose(1, 2), sent_g, cls_g
        return finish

    def _report(self, w0, w1, s0, s1, cl, tid, iid, lc, wi):
        """The logged terms (and the objective) in one launch."""
        with torch.no_grad():
            _, report = K.loss_mix(
                (w0, w1, s0, s1, cl, tid, iid),
                [(1, 1, 1, 1, lc, wi, wi),                            # objective
                 (1, 1, 1, 1, 0, 0, 0),                               # damsm
                 (0, 0, 0, 0, 1, 0, 0),                               # clip
                 (0, 0, 0, 0, 0, wi, wi)])                            # ident
        return {"damsm": report[0], "clip": report[1], "ident": report[2]}

    def _finish(self, w0, w1, s0, s1, cl, tid, iid, lc, wi, pending, groups=None):
        ctx = self.ctx
        out = self._report(w0, w1, s0, s1, cl, tid, iid, lc, wi)
        ctx.wait_grads(pending)
        ctx.reduce_grads(self.head_params)
        self.optimizer.step(groups)
        return out

    def _gather_text(self, words, sent, class_ids):
        """(words, sent, class ids) of the global batch in one all-gather.
        Words that carry the word<->region kernels' operand rows (TextHeading
        in bf16 / fp16 mode) travel as those rows + norms -- bf16 / fp16
        [t_pad, 256] per caption, about half the fp32 words' bytes -- and the
        gathered words are rows-only (kernels.rows_only_words): the DP step
        then re-prepares nothing.  Otherwise the fp32 words themselves."""
        ctx = self.ctx
        words_bt = words.transpose(1, 2)               # [B, T, 256] storage
        f16 = self.args.precision == "fp16"
        pre = K.attached_rows(words_bt, f16, scale=K.LOG2E) \
            if ctx.active and K.wr_rows_path(self.args.precision, words.shape[2],
                                             self.args.en_type == "BERT") else None
        if pre is not None:
            rows, norms = pre
            rows_g, norms_g, sent_g, cls_g = ctx.gather_text(rows, norms, sent, class_ids)
            return K.rows_only_words(rows_g, norms_g, words.shape[2], f16), sent_g, cls_g
        words_g, sent_g, cls_g = ctx.gather_text(words_bt, sent, class_ids)
        return words_g.transpose(1, 2), sent_g, cls_g

    def _identity(self, sent, img_features, class_ids, ctx):
        """(focal(text_cls(sent)), focal(image_cls(img))): one launch per
        direction for both heads (kernels.IdentityHeads; with a process group
        one all-reduce of the two NLL sums gives the global-batch focal
        factor), else the per-head path."""
        tc, ic = self.text_cls, self.image_cls
        if (sent.shape[0] <= 128 and tc.weight.shape == ic.weight.shape
                and tc.m == ic.m and tc.easy_margin == ic.easy_margin):
            return K.identity_heads(sent, tc, img_features, ic, class_ids, self.ident_loss.gamma,
                                    group=ctx.group if ctx.active else None,
                                    n_global=ctx.n_global)
        return K.focal_ce_multi(
            [(tc(sent, class_ids), class_ids), (ic(img_features, class_ids), class_ids)],
            self.ident_loss.gamma, ctx.group if ctx.active else None, ctx.n_global)

    def _weights(self, values, device):
        """Constant device scalars (the loss terms' weights, cached)."""
        cache = self.__dict__.setdefault("_wcache", {})
        key = (tuple(values), device)
        if key not in cache:
            cache[key] = tuple(torch.full((), float(v), device=device) for v in values)
        return cache[key]

    def _labels(self, n, device):
        lab = getattr(self, "_lab", None)
        if lab is None or lab.numel() != n or lab.device != device:
            lab = self._lab = torch.arange(n, device=device)
        return lab


class TrainLSTM(Train):
    """Stage-1 LSTM trainer step (src/train_encoders_lstm.py:236-314).

    The reference also steps an Adam on the text encoder (:178-181), but the
    encoder runs under no_grad (utils/dataset_utils.py:25-33), so that step
    never changes it; the text side here is frozen input as for BERT."""

    _forks = False      # one linear stream (step() below)

    def __init__(self, args, device, ctx=None):
        args.en_type = "LSTM"
        super().__init__(args, device, ctx)
        self.clip_loss = ClipLoss()

    def step(self, batch):
        args, ctx = self.args, self.ctx
        g, local, words, sent, class_ids, cap_lens = batch
        b = g.shape[0]
        ctx.set_batch(b)
        args.dist = ctx
        words_g, sent_g, cls_g, lens_g = ctx.gather_text(words.transpose(1, 2), sent,
                                                         class_ids, cap_lens)
        words_g = words_g.transpose(1, 2)
        labels = self._labels(ctx.n_global, g.device)

        img_features, words_features = self.image_head(g, local)
        self.optimizer.zero_grad(set_to_none=True)
        # :260-266: damsm = w0 + w1 (sent_loss is computed there and discarded)
        w0, w1, _ = words_loss(words_features, words_g, labels, lens_g, cls_g, b, args)
        tid, iid = K.focal_ce_multi(                               # :272-282
            [(self.text_cls(sent, class_ids), class_ids),
             (self.image_cls(img_features, class_ids), class_ids)],
            self.ident_loss.gamma, ctx.group if ctx.active else None, ctx.n_global)
        cl = self.clip_loss(sent_g, img_features, args)            # :288-291
        wi = float(args.lambda_id)
        total, report = K.loss_mix(
            (w0, w1, cl, tid, iid),
            [(1, 1, args.lambda_clip, wi, wi),                     # objective
             (1, 1, 0, 0, 0),                                      # damsm
             (0, 0, args.lambda_clip, 0, 0),                       # clip (logged x lambda)
             (0, 0, 0, wi, wi)])                                   # ident
        total.backward()
        ctx.reduce_grads(self.params)
        self.optimizer.step()
        return {"damsm": report[0], "clip": report[1], "ident": report[2]}


class Fusion:
    """Stage-2 FCFM trainer step (src/fusion_bert.py)."""

    def __init__(self, args, device, ctx=None):
        self.args = args
        self.ctx = ctx or DistContext()
        self.image_head = ImageHeading(args).to(device)
        self.fusion_net = Working(args.aux_feat_dim_per_granularity).to(device)
        self.metric_fc = ArcMarginProduct(640, args.num_classes, s=30, m=0.5).to(device)
        for m in (self.image_head, self.fusion_net, self.metric_fc):
            set_precision(m, args.precision)
        self.params = [p for m in (self.image_head, self.fusion_net, self.metric_fc)
                       for p in m.parameters()]
        self.ctx.broadcast_params(self.params)
        self.criterion = FocalLoss(gamma=2)                        # :92-96
        # :119-130 SGD for the classifier, :137-139 Adam for head + fusion net
        self.optimizer = FusedOptimizer([
            sgd_group(self.metric_fc.parameters(), lr=0.1, weight_decay=5e-4),
            adam_group(list(self.image_head.parameters()) + list(self.fusion_net.parameters()),
                       lr=args.lr_head, weight_decay=5e-5)])

    def step(self, batch):
        g, local, words, sent, class_ids = batch
        ctx = self.ctx
        ctx.set_batch(g.shape[0])
        words = words.requires_grad_()                             # :211-212
        sent = sent.requires_grad_()
        img_feats, local_feats = self.image_head(g, local)         # :220
        output = self.fusion_net(local_feats, words, img_feats, sent)   # :153
        output = self.metric_fc(output, class_ids)                 # :224
        self.optimizer.zero_grad(set_to_none=True)
        # :232; under DP the focal factor of the global-batch mean CE (one
        # all-reduce of the NLL sums), gradients summed over ranks
        loss, = K.focal_ce_multi([(output, class_ids)], self.criterion.gamma,
                                 ctx.group if ctx.active else None, ctx.n_global)
        loss.backward()
        ctx.reduce_grads(self.params)
        self.optimizer.step()
        return {"loss": loss.detach()}


class GraphedStep:
    """A whole train step (forward, backward, optimiser) captured as HIP
    graphs: one graph on a single GPU; with a process group, a chain of graphs
    cut at the step's collectives (text all-gather, one column-partial
    all-gather per contrastive loss, the gradient all-reduce), which replay in
    order with the collectives between them (dist.StepCapture).  The host
    launches a few graphs per step instead of ~370 kernels.

    The batch tensors are static: copy the next batch into them (``load``)
    before each replay.
    """

    def __init__(self, trainer, batch, warmup=3):
        self.batch = batch
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                trainer.step(batch)
        torch.cuda.current_stream().wait_stream(side)
        self.capture = StepCapture()
        self.out = self.capture.capture(trainer.step, batch)

    def load(self, batch):
        for dst, src in zip(self.batch, batch):
            if dst is not src:
                dst.copy_(src, non_blocking=True)

    def step(self, batch=None):
        if batch is not None:
            self.load(batch)
        self.capture.replay()
        return self.out
