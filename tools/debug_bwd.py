"""Debug: bounded bf16 word-region backward vs the oracle for several caption
chunk sizes K (TGFR_BWD_BLOCKS); prints NaN counts per region tile."""
import os
import sys

import torch

sys.path.insert(0, ".")
from oracle import tgfr_oracle as O  # noqa: E402
from text_guided_face_recognition_amd import kernels as K  # noqa: E402


def unit(x):
    return x / x.norm(dim=-1, keepdim=True)


def run(b_img, b_cap, nw, blocks):
    os.environ["TGFR_BWD_BLOCKS"] = str(blocks)
    torch.manual_seed(3)
    r = unit(torch.randn(b_img, 14, 14, 256)).permute(0, 3, 1, 2)
    w = unit(torch.randn(b_cap, nw, 256)).transpose(1, 2)
    ro = r.clone().requires_grad_()
    _, _, _, ref = O.words_loss(ro, w, None, None, nw, 4.0, 5.0, 10.0, batch_size=b_cap)
    probe = torch.randn(b_img, b_cap)
    (ref * probe).sum().backward()
    rg = r.cuda().requires_grad_()
    lg = K.word_region_logits(rg, K.words_view(w.cuda(), nw),
                              torch.full((b_cap,), nw, dtype=torch.int32), 4.0, 5.0, 10.0,
                              mode="bf16", bounded=True)
    (lg * probe.cuda()).sum().backward()
    g = rg.grad.cpu().permute(0, 2, 3, 1).reshape(b_img, 196, 256)
    gr = ro.grad.permute(0, 2, 3, 1).reshape(b_img, 196, 256)
    nan = ~torch.isfinite(g)
    tiles = [int(nan[:, 32 * j:32 * j + 32].sum()) for j in range(7)]
    err = ((g - gr).abs().max() / gr.abs().max()).item()
    chunks = K.bwd_chunks(b_img, b_cap)
    print(f"b_img={b_img} b_cap={b_cap} T={nw} chunks={chunks} K={-(-b_cap // chunks)} "
          f"logit_err={(lg.detach().cpu() - ref.detach()).abs().max():.3e} "
          f"nan_per_tile={tiles} grad_err={err:.3e}", flush=True)


for blocks in (256, 32, 16, 8):
    run(4, 8, 30, blocks)
run(16, 16, 22, 256)
