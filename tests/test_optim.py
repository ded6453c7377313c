"""The one-launch optimiser step (tgfr_optim_step, optim.FusedOptimizer)
against torch.optim.Adam / torch.optim.SGD (for-loop implementations, fp32) on
the same parameters and gradients, eagerly and replayed from a HIP graph."""
import pytest
import torch

from text_guided_face_recognition_amd.optim import FusedOptimizer, adam_group, sgd_group

# shapes of the stage-1 trainer's tensors plus ragged sizes (scalar tail path)
SHAPES = [(256, 512), (256,), (128, 256, 1, 1), (256, 14, 14), (7,), (3, 5), (4500, 256)]


def _groups(params, fused, cfg):
    a, s = params[:4], params[4:]
    if cfg == "stage1":
        if fused:
            return [adam_group(a, lr=2e-4, betas=(0.5, 0.999)),
                    sgd_group(s, lr=0.1, momentum=0.9, weight_decay=5e-5)]
        return [torch.optim.Adam(a, lr=2e-4, betas=(0.5, 0.999), foreach=False),
                torch.optim.SGD(s, lr=0.1, momentum=0.9, weight_decay=5e-5, foreach=False)]
    # stage 2 (src/fusion_bert.py:119-139): plain SGD with decay, Adam with decay
    if fused:
        return [sgd_group(s, lr=0.1, weight_decay=5e-4),
                adam_group(a, lr=2e-4, weight_decay=5e-5)]
    return [torch.optim.SGD(s, lr=0.1, weight_decay=5e-4, foreach=False),
            torch.optim.Adam(a, lr=2e-4, weight_decay=5e-5, foreach=False)]


def _setup(dev, cfg, seed=0):
    gen = torch.Generator().manual_seed(seed)
    init = [torch.randn(s, generator=gen) * 0.1 for s in SHAPES]
    grads = [[torch.randn(s, generator=gen) for s in SHAPES] for _ in range(4)]
    mine = [p.to(dev).requires_grad_() for p in init]
    ref = [p.to(dev).clone().requires_grad_() for p in init]
    return mine, ref, grads


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["stage1", "stage2"])
def test_group_subsets_match_one_step(gpu, cfg):
    """step(groups=[SGD group]) on a second stream, then step(groups=[Adam
    group]) on the current one (the forked trainer step's split) updates every
    parameter exactly as one full step, and counts one step."""
    mine, ref, grads = _setup(gpu, cfg)
    opt = FusedOptimizer(_groups(mine, True, cfg))
    full = FusedOptimizer(_groups(ref, True, cfg))
    sgd_i = [i for i, g in enumerate(opt._all_groups) if g["kind"] != 0][0]
    adam_i = 1 - sgd_i
    side = torch.cuda.Stream()
    for gs in grads:
        for p, q, g in zip(mine, ref, gs):
            p.grad = g.to(gpu)
            q.grad = g.to(gpu)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            opt.step(groups=[sgd_i])
        opt.step(groups=[adam_i])
        torch.cuda.current_stream().wait_stream(side)
        full.step()
        for p, q in zip(mine, ref):
            assert torch.equal(p, q)
    assert opt.step_count == len(grads)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", ["stage1", "stage2"])
def test_fused_matches_torch(gpu, cfg):
    mine, ref, grads = _setup(gpu, cfg)
    opt = FusedOptimizer(_groups(mine, True, cfg))
    topts = _groups(ref, False, cfg)
    for gs in grads:
        opt.zero_grad()
        for o in topts:
            o.zero_grad()
        for p, q, g in zip(mine, ref, gs):
            p.grad = g.to(gpu)
            q.grad = g.to(gpu)
        opt.step()
        for o in topts:
            o.step()
        for p, q in zip(mine, ref):
            err = ((p - q).abs().max() / q.abs().max()).item()
            assert err < 1e-6, err
    assert opt.step_count == len(grads)


@pytest.mark.gpu
def test_graph_replay_matches_torch(gpu):
    """Captured once (grads in static buffers), replayed: the device step count
    gives every replay its own bias corrections / first-step momentum."""
    mine, ref, grads = _setup(gpu, "stage1", seed=1)
    opt = FusedOptimizer(_groups(mine, True, "stage1"))
    topts = _groups(ref, False, "stage1")
    static = [torch.zeros(s, device=gpu) for s in SHAPES]
    for p, g in zip(mine, static):
        p.grad = g
    # warm the library on the capture stream, then undo that step
    snap = [p.detach().clone() for p in mine]
    opt.step()
    torch.cuda.synchronize()
    with torch.no_grad():
        for p, s in zip(mine, snap):
            p.copy_(s)
        for st in opt.state.values():
            for b in st:
                b.zero_()
        opt.counters.zero_()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        opt.step()
    # capture ran nothing: state untouched
    assert opt.step_count == 0
    for gs in grads:
        for g, h in zip(static, gs):
            g.copy_(h)
        graph.replay()
        for o in topts:
            o.zero_grad()
        for q, g in zip(ref, gs):
            q.grad = g.to(gpu)
        for o in topts:
            o.step()
    torch.cuda.synchronize()
    for p, q in zip(mine, ref):
        err = ((p - q).abs().max() / q.abs().max()).item()
        assert err < 1e-6, err
    assert opt.step_count == len(grads)


def test_rejects_host_tensors():
    p = torch.zeros(8, requires_grad=True)
    opt = FusedOptimizer([adam_group([p])])
    p.grad = torch.ones(8)
    with pytest.raises(RuntimeError, match="device tensors"):
        opt.step()


def test_limits():
    ps = [torch.zeros(4, requires_grad=True) for _ in range(49)]
    with pytest.raises(ValueError):
        FusedOptimizer([adam_group(ps)])
    with pytest.raises(ValueError):
        FusedOptimizer([adam_group([torch.zeros(4, dtype=torch.float64)])])


@pytest.mark.gpu
def test_lr_schedule_between_graph_replays(gpu):
    """The reference's schedules (ExponentialLR(0.98) on the head every epoch,
    the classifier SGD lr cut 10x at epochs 3 and 8,
    src/train_encoders_bert.py:225, :406-410) applied between replays of ONE
    captured step match torch.optim + torch.optim.lr_scheduler."""
    mine, ref, grads = _setup(gpu, "stage1", seed=2)
    opt = FusedOptimizer(_groups(mine, True, "stage1"))
    adam, sgd = _groups(ref, False, "stage1")
    sched = torch.optim.lr_scheduler.ExponentialLR(adam, gamma=0.98)
    static = [torch.zeros(s, device=gpu) for s in SHAPES]
    for p, g in zip(mine, static):
        p.grad = g
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph):
            opt.step()
    torch.cuda.current_stream().wait_stream(side)
    for epoch, gs in enumerate(grads * 3):
        for g, h in zip(static, gs):
            g.copy_(h)
        graph.replay()
        for o in (adam, sgd):
            o.zero_grad()
        for q, g in zip(ref, gs):
            q.grad = g.to(gpu)
        adam.step()
        sgd.step()
        # end of "epoch": schedules advance on both sides
        sched.step()
        opt.scale_lr(0, 0.98)
        if epoch in (3, 8):
            for pg in sgd.param_groups:
                pg["lr"] *= 0.1
            # the reference's own pattern (src/train_encoders_bert.py:408-410)
            for pg in opt.param_groups[1:]:
                pg["lr"] *= 0.1
        assert abs(opt.get_lr(0) - adam.param_groups[0]["lr"]) < 1e-12
        assert abs(opt.get_lr(1) - sgd.param_groups[0]["lr"]) < 1e-12
    torch.cuda.synchronize()
    for p, q in zip(mine, ref):
        err = ((p - q).abs().max() / q.abs().max()).item()
        assert err < 1e-5, err


def test_param_groups_lr_assignment_reaches_the_kernel():
    """``g['lr'] = x`` on param_groups (the reference's classifier lr cut,
    src/train_encoders_bert.py:408-410) changes the device lr factor the kernel
    reads, not only the reported value; indices follow the caller's list even
    with an empty group; a rejected set_lr leaves the state unchanged."""
    a = [torch.zeros(4, requires_grad=True)]
    s = [torch.zeros(3, requires_grad=True)]
    z = [torch.zeros(2, requires_grad=True)]
    opt = FusedOptimizer([adam_group(a, lr=2e-4), adam_group([], lr=1.0),
                          sgd_group(s, lr=0.1), sgd_group(z, lr=0.0)])
    groups = opt.param_groups
    assert len(groups) == 4 and groups[2]["lr"] == 0.1
    for g in groups[2:3]:
        g["lr"] *= 0.1
    assert abs(opt.get_lr(2) - 0.01) < 1e-12
    assert abs(opt.lr_scale[1].item() - 0.1) < 1e-7          # internal slot of group 2
    assert abs(groups[2]["lr"] - 0.01) < 1e-12
    opt.scale_lr(0, 0.98)
    assert abs(opt.param_groups[0]["lr"] - 2e-4 * 0.98) < 1e-12
    assert abs(opt.lr_scale[0].item() - 0.98) < 1e-7
    groups[1]["lr"] = 0.5                                     # empty group: host value only
    assert opt.get_lr(1) == 0.5
    before = opt.lr_scale.clone()
    with pytest.raises(ValueError):
        groups[3]["lr"] = 1e-3                                # base lr 0 cannot be rescaled
    assert opt.get_lr(3) == 0.0 and groups[3]["lr"] == 0.0
    assert torch.equal(before, opt.lr_scale)
    with pytest.raises(ValueError):
        groups[0]["betas"] = (0.9, 0.9)
