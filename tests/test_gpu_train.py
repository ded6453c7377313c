"""GPU: the stage-1 and stage-2 train steps run end to end, and the HIP-graph
replay of a step is numerically identical to eager execution."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _build(dev, precision="fp32", cls="Train", b=16):
    from text_guided_face_recognition_amd import train as T
    from text_guided_face_recognition_amd.config import make_args
    torch.manual_seed(123)
    args = make_args(batch_size=b, num_classes=200, precision=precision, bert_words_num=24)
    return getattr(T, cls)(args, dev)


def _batch(dev, b=16, nw=22):
    from text_guided_face_recognition_amd.train import synthetic_batch
    return synthetic_batch(b, nw, dev, seed=5, n_ids=200)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_graph_replay_matches_eager(gpu, precision):
    from text_guided_face_recognition_amd.train import GraphedStep
    batch = _batch(gpu)
    eager = _build(gpu, precision)
    graphed = _build(gpu, precision)
    outs_e = [eager.step(batch) for _ in range(5)]
    gs = GraphedStep(graphed, tuple(t.clone() for t in batch), warmup=3)
    outs_g = [{k: v.clone() for k, v in gs.step().items()}]
    outs_g += [{k: v.clone() for k, v in gs.step().items()}]
    torch.cuda.synchronize()
    # graphed trainer took 3 warm-up + 2 replayed steps == eager's 5 steps
    for k in outs_e[-1]:
        torch.testing.assert_close(outs_g[-1][k], outs_e[-1][k], rtol=1e-5, atol=1e-5)
    pe = dict(eager.image_head.named_parameters())
    for n, p in graphed.image_head.named_parameters():
        torch.testing.assert_close(p, pe[n], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("fork", ["1", "2"])
def test_forked_step_matches_linear(gpu, monkeypatch, fork):
    """The forked single-process step (the g' branch, and with TGFR_FORK=2
    TextHeading, on a side stream) runs the same kernels on the same inputs
    as the linear step: losses and parameters after three steps agree to the
    atomics-order noise of the split reductions."""
    batch = _batch(gpu)
    monkeypatch.setenv("TGFR_FORK", "0")
    lin = _build(gpu, "bf16")
    monkeypatch.setenv("TGFR_FORK", fork)
    frk = _build(gpu, "bf16")
    assert lin._side is None and frk._side is not None
    outs_l = [lin.step(batch) for _ in range(3)]
    outs_f = [frk.step(batch) for _ in range(3)]
    torch.cuda.synchronize()
    for k in outs_l[-1]:
        torch.testing.assert_close(outs_f[-1][k], outs_l[-1][k], rtol=1e-5, atol=1e-5)
    pl = dict(lin.image_head.named_parameters())
    for n, p in frk.image_head.named_parameters():
        torch.testing.assert_close(p, pl[n], rtol=1e-5, atol=1e-6)
    # the classifiers: updated on the side stream by their own (Adam-free)
    # optimiser launch in the forked step -- parameters and SGD momentum
    # buffers must match the linear step's single launch
    for mod in ("image_cls", "text_cls"):
        ml, mf = getattr(lin, mod), getattr(frk, mod)
        for (n, p), q in zip(mf.named_parameters(), ml.parameters()):
            torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6, msg=f"{mod}.{n}")
            sf, sl = frk.optimizer.state[p], lin.optimizer.state[q]
            assert len(sf) == len(sl) >= 1, (mod, n)
            for a, b in zip(sf, sl):
                torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6, msg=f"{mod}.{n} state")


def test_fusion_step(gpu):
    tr = _build(gpu, cls="Fusion", b=8)
    batch = _batch(gpu, b=8)
    first = tr.step(batch)["loss"].item()
    for _ in range(5):
        last = tr.step(batch)["loss"].item()
    assert torch.isfinite(torch.tensor([first, last])).all()
    assert last < first        # the FCFM head learns the fixed batch


def test_plain_torch_graph_capture(gpu):
    """The standard PyTorch recipe -- torch.cuda.graph on its own capture
    stream, no dist.StepCapture -- captures kernels that use the in-launch
    counters (the single-rank contrastive CE's last-arriver loss block): the
    counter buffer is made inside the capture and re-zeroed by the graph, and
    replays reproduce eager losses and gradients."""
    import torch.nn.functional as F  # noqa: F401
    from text_guided_face_recognition_amd import kernels as K
    torch.manual_seed(2)
    unit = lambda x: x / x.norm(dim=-1, keepdim=True)  # noqa: E731
    r = unit(torch.randn(12, 14, 14, 256, device=gpu)).permute(0, 3, 1, 2).requires_grad_()
    w = unit(torch.randn(12, 30, 256, device=gpu))
    lens = torch.full((12,), 30, dtype=torch.int32, device=gpu)

    def step():
        r.grad = None
        logits = K.word_region_logits(r, w, lens, 4.0, 5.0, 10.0, mode="bf16", bounded=True)
        l0, l1 = K.contrastive_ce(logits)
        (l0 + l1).backward()
        return (l0 + l1).detach()
    ref = step()
    ref_g = r.grad.clone()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        step()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    r.grad = None
    with torch.cuda.graph(g):
        out = step()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert torch.equal(r.grad, ref_g)
