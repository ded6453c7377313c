"""Time the word-region kernels at BASELINE config 2 (B=64, T=30) with HIP events."""
import sys
import torch
import torch.nn.functional as F
sys.path.insert(0, ".")
from text_guided_face_recognition_amd import kernels as K


def unit(x):
    return x / x.norm(dim=-1, keepdim=True)


def main(b=64, nw=30, mode="fp32", iters=20, bounded=True):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    r = unit(torch.randn(b, 14, 14, 256, device=dev)).permute(0, 3, 1, 2).requires_grad_()
    w = unit(torch.randn(b, nw, 256, device=dev))
    lens = torch.full((b,), nw, dtype=torch.int32, device=dev)
    labels = torch.arange(b, device=dev)

    def step():
        logits = K.word_region_logits(r, w, lens, 4.0, 5.0, 10.0, mode=mode, bounded=bounded)
        loss = F.cross_entropy(logits, labels) + F.cross_entropy(logits.t(), labels)
        loss.backward()
        return loss
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        step()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    flop = 10 * 196 * 256 * nw * b * b
    from text_guided_face_recognition_amd._hip import KernelTimer
    with KernelTimer(replay=("tgfr_wr_fwd", "tgfr_wr_bwd")) as kt:
        for _ in range(5):
            step()
    fwd, bwd = kt.replayed["tgfr_wr_fwd"], kt.replayed["tgfr_wr_bwd"]
    f_tf = 4 * 196 * 256 * nw * b * b / fwd / 1e9
    b_tf = 6 * 196 * 256 * nw * b * b / bwd / 1e9
    print(f"mode={mode} bounded={bounded} B={b} T={nw}: {ms:.3f} ms/step  {flop / ms / 1e9:.1f} TFLOP/s algorithmic"
          f" | fwd {fwd * 1000:.1f} us ({f_tf:.0f} TF)  bwd {bwd * 1000:.1f} us ({b_tf:.0f} TF)")


if __name__ == "__main__":
    if "--bf16-only" in sys.argv:
        rest = [a for a in sys.argv[1:] if not a.startswith("--")]
        main(b=int(rest[0]) if rest else 64, nw=int(rest[1]) if len(rest) > 1 else 30,
             mode="bf16", iters=3)
        sys.exit(0)
    if "--unbounded" in sys.argv:
        main(mode="bf16", bounded=False)
        main(b=128, mode="bf16", bounded=False)
        sys.exit(0)
    for mode in ("fp32", "bf16"):
        main(mode=mode)
        main(b=256, mode=mode)
