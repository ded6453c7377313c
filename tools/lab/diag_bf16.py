"""Diagnose the bf16 word-region forward's logit error on a reference fixture:
compare the kernel's per-token stats {Z, n, |C|, cos} with a float64 model of
the same bf16 arithmetic (operands rounded as the kernel rounds them)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from text_guided_face_recognition_amd import kernels as K  # noqa: E402

L2E = 1.4426950408889634


def main(name="words_loss_bert_b4_t30"):
    z = np.load(f"tests/golden/{name}.npz")
    dev = torch.device("cuda")
    r = torch.from_numpy(z["img_features"])
    w = torch.from_numpy(z["words_emb"])
    nw = int(z["bert_words_num"]) - 2
    b = r.shape[0]
    regions = K.regions_view(r.to(dev))
    words = K.words_view(w.to(dev), nw)
    lens = torch.full((b,), nw, dtype=torch.int32, device=dev)
    r_hi, _, r_norm = K.prep_rows(regions.float(), K.NREG, K.RPAD, want_norms=True)
    w_hi, _, w_norm = K.prep_rows(words.float(), nw, K.TPAD, lens=lens, want_norms=True,
                                  scale=L2E)
    logits = torch.empty(b, b, device=dev)
    stats = torch.empty(b, b, K.TPAD, 4, device=dev)
    c_hi = torch.empty(b, b, 32, K.TPAD, 8, dtype=torch.int16, device=dev)
    for bounded in (1, 0):
        K.call("tgfr_wr_fwd", K.ptr(r_hi), None, K.ptr(w_hi), None, K.ptr(w_norm),
               K.ptr(r_norm), K.ptr(lens), b, b, 0, 4.0, 5.0, 10.0, 1e-8, K.ptr(logits), b,
               K.ptr(stats), K.ptr(c_hi), None, None, 0, bounded, K.TPAD, 0, K._hip.stream())
        torch.cuda.synchronize()
        ref = z["logits"]
        print(f"bounded={bounded} max |logit err| {np.abs(logits.cpu().numpy() - ref).max():.3e}")
        st = stats.cpu().double().numpy()
        # float64 model of the bf16 arithmetic
        R = torch.from_numpy(r_hi.cpu().numpy().view(np.uint16).astype(np.uint32) << 16)
        R = R.view(torch.float32).double()[:, :196]
        Wp = torch.from_numpy(w_hi.cpu().numpy().view(np.uint16).astype(np.uint32) << 16)
        Wp = Wp.view(torch.float32).double()[:, :nw] / L2E
        bf = lambda x: x.float().to(torch.bfloat16).double()  # noqa: E731
        worst = {}
        for bi in range(b):
            for i in range(b):
                S = R[bi] @ Wp[i].T
                A1 = torch.softmax(S, 1)
                E = torch.exp(4 * A1)
                Eb = bf(E)
                Z = Eb.sum(0)
                C = Eb.T @ R[bi]
                n = (E * S).sum(0) / Z
                cn = C.norm(dim=1) / Z
                u = torch.from_numpy(w_norm.cpu().numpy()[i, :nw]).double()
                cos = n / (u * cn)
                for k, (m, g) in enumerate([(Z, st[bi, i, :nw, 0]), (n, st[bi, i, :nw, 1]),
                                             (cn, st[bi, i, :nw, 2]), (cos, st[bi, i, :nw, 3])]):
                    e = (np.abs(m.numpy() - g) / np.maximum(np.abs(m.numpy()), 1e-12)).max()
                    worst[k] = max(worst.get(k, 0), e)
        print("  worst relative stat error vs the model: Z %.2e n %.2e |C| %.2e cos %.2e" %
              tuple(worst[k] for k in range(4)))


if __name__ == "__main__":
    main(*sys.argv[1:])
