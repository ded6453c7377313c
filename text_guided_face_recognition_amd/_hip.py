"""ctypes binding of libtgfr_hip.so (include/tgfr.h).

The library is loaded after torch so that its NEEDED libamdhip64.so.7 resolves
to the HIP runtime torch already mapped (same SONAME): one runtime per
process, so torch's streams and device pointers are valid in the kernels.
There is no fallback: if the library cannot be built or a call fails, this
module raises.  A library whose source stamp does not match the tree (or a
missing one) is rebuilt from csrc/ before it is mapped (build.stale), so the
kernels that run are always the ones in the tree.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must be imported before the library is mapped)

from . import build as _build

LIB = _build.LIB

_lib = None

P = C.c_void_p
I = C.c_int
L = C.c_longlong
F = C.c_float

# name -> argtypes (restype int unless noted)
SIGNATURES = {
    "tgfr_version": [],
    "tgfr_prep_rows": [P, L, L, L, I, I, I, I, P, F, P, P, P, P],
    "tgfr_prep_rows_f16": [P, L, L, L, I, I, I, I, P, F, P, P, P],
    "tgfr_wr_fwd": [P, P, P, P, P, P, P, I, I, I, F, F, F, F, P, I, P, P, P, P, P, I, I, I, I, P,
                    P],
    "tgfr_wr_guard": [P, I, P, I, P, P],
    "tgfr_wr_bwd_tok": [P, P, P, P, I, I, F, F, F, F, P, I, I, I, P, P, P],
    "tgfr_wr_bwd_tok_ce": [P, P, P, P, I, I, F, F, F, F, P, I, I, F, P, P, P, P, F, F, I, I, P,
                           P, P],
    "tgfr_wr_bwd_ws": [I, I, I, I, I, P],
    "tgfr_wr_bwd": [P, P, P, P, I, I, F, P, P, P, P, P, L, L, L, P, I, I, I, P, P, P],
    "tgfr_wr_lds_bytes": [I],
    "tgfr_cos_logits": [P, L, P, L, I, I, I, I, F, F, I, P, I, P, L, P],
    "tgfr_cos_logits_bwd": [P, L, L, P, L, P, L, I, I, I, I, F, F, P, L, P],
    "tgfr_ce_stats": [P, L, I, I, P, P, P, P, I, F, P, P, P],
    "tgfr_ce_loss": [P, L, I, I, F, P, P, P, P],
    "tgfr_col_lse_combine": [P, I, L, I, P, P],
    "tgfr_focal_global": [I, P, I, L, I, I, F, F, P, P, P, P, P],
    "tgfr_ce_grad": [P, L, I, I, I, F, P, P, P, P, F, F, P, L, P],
    "tgfr_bgemm": [P, L, L, L, P, L, L, L, P, L, L, L, I, I, I, I, F, I, P, I, I, P, P, I, P],
    "tgfr_attn_softmax": [P, P, P, L, I, L, F, P],
    "tgfr_l2norm_rows": [P, L, I, I, F, P, L, P, P],
    "tgfr_l2norm_rows_bwd": [P, L, P, L, P, I, I, F, P, L, P],
    "tgfr_arc_margin": [P, P, I, I, F, F, I, P, P],
    "tgfr_arc_margin_bwd": [P, P, P, I, I, F, F, I, P, P],
    "tgfr_focal_ce": [P, I, I, P, F, P, P, P, P],
    "tgfr_focal_ce_bwd": [P, I, I, P, F, P, P, P, P],
    "tgfr_attn_softmax_bwd": [P, P, P, L, I, L, F, P],
    "tgfr_attn_fwd": [P, P, P, L, L, I, I, F, P, L, L, P, P],
    "tgfr_linear_bf16out": [P, L, I, I, P, L, P, I, P, L, P],
    "tgfr_attn_bwd_ws": [I, I, P],
    "tgfr_attn_small_fwd": [P, L, L, P, L, L, I, I, I, I, I, I, F, P, L, L, P, P],
    "tgfr_attn_small_bwd": [P, L, L, P, L, L, I, I, I, I, I, I, F, P, P, L, L, P, L, L, P, L, L,
                            P],
    "tgfr_attn_bwd": [P, P, P, L, L, I, I, F, P, P, L, L, P, P, P, P, L, L, P, P],
    "tgfr_ln_ws_floats": [I, L, I, I, P],
    "tgfr_loss_mix": [I, P, I, P, P, P],
    "tgfr_bn_fwd_cl": [P, I, I, I, F, F, I, P, P, P, P, P, P, P],
    "tgfr_bn_fold": [P, P, I, I, P, P, P, P, P],
    "tgfr_bn_unfold": [P, P, P, I, I, P, P, P, P, P, P, P, P],
    "tgfr_loss_mix_bwd": [P, I, P, P, P],
    "tgfr_bias_grad": [P, L, I, I, P, L, P, L, P, P, P, P],
    "tgfr_ln_fwd": [P, I, L, P, P, F, I, P, P, P],
    "tgfr_ln_bwd": [P, P, I, L, P, I, P, P, P, P, P],
    "tgfr_pair_cosine": [P, L, P, L, I, I, F, P, P],
    "tgfr_func_attention_fwd": [P, L, L, L, P, L, L, L, I, I, I, I, F, P, L, L, L, P, P, P],
    "tgfr_func_attention_bwd": [P, L, L, L, P, L, L, L, P, L, L, L, P, I, I, I, I, F, P, P, P,
                                P, P],
    "tgfr_tail_pack_elems": [],
    "tgfr_tail_pack": [P, P, P, P, P],
    "tgfr_tail_fwd": [P, L, I, P, P, P, P, F, P, L, P, P, P, P, P, P, I, I, I, P],
    "tgfr_tail_bwd": [P, L, P, L, P, I, F, P, P, P, P, L, P, P, P, P],
    "tgfr_tail_dw_ws": [I, P],
    "tgfr_dw_bf16_ws": [I, I, I, P],
    "tgfr_dw_bf16": [P, P, I, I, I, I, P, P, P, P],
    "tgfr_tail_dw": [P, P, P, P, P, P, I, P, P, P, P, P, P, P, P],
    "tgfr_optim_step": [P, I, P, I, P, P, P],
    "tgfr_arc_fwd": [P, L, I, I, P, L, I, P, F, F, I, F, P, P, P, P, P, P],
    "tgfr_arc_bwd": [P, P, P, P, P, L, P, I, I, I, F, F, I, F, P, L, P, P, P],
    "tgfr_arc_bwd_ws": [I, I, I, P],
    "tgfr_text_pack_bytes": [I, P],
    "tgfr_text_pack": [P, P, I, P],
    "tgfr_text_heading_ws": [I, I, P],
    "tgfr_text_heading": [P, I, I, P, P, P, P, L, L, P, L, P, P, I, F, I, I, P],
    "tgfr_sent_global": [P, L, P, L, I, P, F, F, F, P, P, P, P, P],
    "tgfr_sent_global_bwd": [P, P, P, P, L, P, L, I, P, F, F, F, P, P, P, P, L, P],
    "tgfr_sent_global_dist_ws": [I, I, P, P, P],
    "tgfr_sent_global_dist_fwd": [P, L, I, P, L, I, P, I, F, F, F, P, P, P, P, P],
    "tgfr_sent_global_dist_loss": [P, I, I, I, F, F, P, P, I, L, F, P, P, P],
    "tgfr_sent_global_dist_bwd": [P, P, P, P, L, I, P, L, I, P, I, F, F, F, F, P, P, P, P, L,
                                  P],
    "tgfr_focal_ce2": [P, P, I, I, P, F, P, P, P, P, P, P],
    "tgfr_arc_fwd_heads": [P, I, I, I, I, F, I, F, P],
    "tgfr_arc_focal_bwd_heads": [P, I, I, I, I, F, I, F, F, P],
    "tgfr_bn_fold3": [P, P, I, I, P, P, P, P, P],
    "tgfr_bn_unfold3": [P, P, P, I, I, P, P, P, P, P, P, P, P],
    "tgfr_fcfm_pack_elems": [],
    "tgfr_maxpool2_cl": [P, I, I, I, I, P, P, P],
    "tgfr_maxpool2_cl_bwd": [P, P, I, I, I, I, P, P],
    "tgfr_bn_bwd_cl": [P, P, P, I, I, I, I, P, P],
    "tgfr_fcfm_pack": [P, P, P],
    "tgfr_fcfm_conv_fwd": [P, L, L, I, P, P, P, P, I, P],
    "tgfr_fcfm_conv_dx": [P, P, I, P, P, L, L, I, P],
    "tgfr_fcfm_conv_dw_ws": [I, P],
    "tgfr_fcfm_conv_dw": [P, L, L, P, P, I, P, P, P, I, P],
    "tgfr_ln_tail_ws": [I, I, P],
    "tgfr_imim_dw_ws": [I, I, I, P],
    "tgfr_imim_dw": [P, P, P, P, P, P, I, P, P, P, P, P, P, P, P, I, I, P, P, P, P],
    "tgfr_imim_dw_ln": [P, P, P, P, P, P, I, P, P, P, P, P, P, P, P, I, I, P, P, P, I, P, P,
                        P, P],
    "tgfr_attn_fwd_ln": [P, P, P, L, L, I, I, F, P, P, P, P],
    "tgfr_ln_tail_fwd_att": [P, I, I, F, P, P, P, P, P, F, P, L, P, P, P, P, P, P, I, I, I, P],
    "tgfr_ln_tail_bwd_att": [P, P, P, I, F, P, P, P, P, I, P, P, P, P, P, P, P, P, P],
    "tgfr_attn_bwd_prepped": [P, P, P, L, L, I, I, F, P, P, P, P, L, L, P, P],
    "tgfr_imim_pack": [P, P, I, I, P, P, P, P, P, P, P, P, P, I, I, P, P, P],
    "tgfr_bn_fwd_cl_bf16": [P, I, I, I, F, F, I, P, P, P, P, P, P, P],
    "tgfr_bn_stats": [P, I, I, I, F, F, I, P, P, P, P, P, P],
    "tgfr_imim_prep": [P, I, I, F, F, I, P, P, P, P, P, P, P, I, I, P, P, P, P, P, P, P, P, P,
                       P, I, I, P, P, P],
    "tgfr_bn_qkv_bf16": [P, I, I, I, P, P, P, P, I, P, P, P],
    "tgfr_linear_bf16io": [P, L, I, I, P, L, P, I, P, L, P],
    "tgfr_tail_pack_ln": [P, P, P, P, P, I, I, P, P, P],
    "tgfr_ln_tail_fwd": [P, I, I, F, P, P, P, P, P, F, P, L, P, P, P, P, P, P, I, I, I, P],
    "tgfr_ln_tail_bwd": [P, P, P, I, F, P, P, P, P, I, P, P, P, P, P, P, P, P, P],
    "tgfr_proj_l2norm_ws": [I, I, P],
    "tgfr_proj_l2norm_fwd": [P, L, I, I, P, L, P, I, F, P, P, L, P, P, P],
    "tgfr_proj_dw": [P, L, P, L, I, I, I, P, L, P, P],
    "tgfr_arc_dx_ws": [I, I, I, P],
    "tgfr_arc_dx": [P, P, L, I, I, I, P, P, F, P, P, P],
}


def lib():
    """The loaded kernel library (raises if it has not been built)."""
    global _lib
    if _lib is None and os.environ.get("TGFR_LIB"):
        # a lab build of the library (tools/lab/variants.py), for A/B timing
        # only: it bypasses the stamp check, so it takes an explicit opt-in
        if os.environ.get("TGFR_LAB") != "1":
            raise RuntimeError("TGFR_LIB names a lab build of the kernel library; set "
                               "TGFR_LAB=1 to load it (A/B timing only)")
        _lib = _bind(C.CDLL(os.environ["TGFR_LIB"], mode=C.RTLD_GLOBAL))
    if _lib is None:
        if _build.stale():
            import sys
            sys.stderr.write(f"[tgfr] {LIB} is missing or stale: building it from csrc/\n")
            try:
                _build.build()
            except Exception as e:  # noqa: BLE001
                raise RuntimeError(f"{LIB} could not be built ({e}); there is no CPU "
                                   "fallback") from e
        _lib = _bind(C.CDLL(LIB, mode=C.RTLD_GLOBAL))
    return _lib


def _bind(handle):
    for name, argtypes in SIGNATURES.items():
        fn = getattr(handle, name, None)
        if fn is None:
            continue
        fn.argtypes = argtypes
        fn.restype = I
    return handle


def exported_symbols():
    return [n for n in SIGNATURES if getattr(lib(), n, None) is not None]


class KernelTimer:
    """Brackets every library call with HIP events on torch's current stream
    (the stream the kernels are launched on) while active.

    replay: entry points whose first call is also re-launched `reps` times
    back to back, bracketed by one pair of events, right after the call
    returns -- while every buffer it was given is still alive -- to measure
    the kernel's own duration without per-call host gaps (the launches are
    idempotent: each rewrites its outputs from unchanged inputs)."""

    active = None

    def __init__(self, replay=(), reps=20):
        self.events = {}
        self.replay = set(replay)
        self.reps = reps
        self.replayed = {}

    def __enter__(self):
        KernelTimer.active = self
        return self

    def __exit__(self, *exc):
        KernelTimer.active = None

    def record(self, name, fn):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        rc = fn()
        e.record()
        self.events.setdefault(name, []).append((s, e))
        if rc == 0 and name in self.replay and name not in self.replayed:
            r0 = torch.cuda.Event(enable_timing=True)
            r1 = torch.cuda.Event(enable_timing=True)
            r0.record()
            for _ in range(self.reps):
                fn()
            r1.record()
            r1.synchronize()
            self.replayed[name] = r0.elapsed_time(r1) / self.reps
        return rc

    def summary(self):
        """name -> (calls, average ms); synchronises."""
        torch.cuda.synchronize()
        out = {}
        for name, evs in self.events.items():
            ms = [s.elapsed_time(e) for s, e in evs]
            out[name] = (len(ms), sum(ms) / len(ms))
        return out


_counters = {}
N_COUNTERS = 1 << 20
_hiprt = None


def _capture_id(stream_handle):
    """The HIP graph capture id of a stream, or None when it is not capturing
    (hipStreamGetCaptureInfo of the runtime torch mapped)."""
    global _hiprt
    if not torch.cuda.is_current_stream_capturing():
        return None
    if _hiprt is None:
        _hiprt = lib()        # dlsym through the library reaches its HIP runtime
        _hiprt.hipStreamGetCaptureInfo.argtypes = [P, C.POINTER(I), C.POINTER(C.c_ulonglong)]
    st, cid = I(0), C.c_ulonglong(0)
    rc = _hiprt.hipStreamGetCaptureInfo(P(stream_handle), C.byref(st), C.byref(cid))
    if rc != 0:
        raise RuntimeError(f"hipStreamGetCaptureInfo failed with code {rc}")
    return int(cid.value) if st.value == 1 else None


def counters(device):
    """Zeroed uint32 words for the kernels' in-launch last-arriver hand-offs,
    one buffer per (device, stream): kernels on one stream run one at a time
    and every kernel leaves the words it used at zero again, so the calls of a
    stream share its buffer, while kernels of different streams never share
    a word.
    A stream's buffer is made on first use.  Made inside a HIP graph capture
    (e.g. plain torch.cuda.graph, whose capture stream is its own), the buffer
    comes from that graph's memory pool and its zeroing is a node of that
    graph, so it is cached for that capture only (keyed by the capture id):
    another capture on the same stream, or eager use of it, makes its own
    zeroed buffer instead of reading words only that graph ever zeroes.
    (dist.StepCapture makes its stream's buffer before capturing, so its
    graphs carry no such node.)"""
    dev = torch.device(device)
    stream = torch.cuda.current_stream(dev)
    key = (dev.index, stream.cuda_stream)
    buf = _counters.get(key)
    if buf is None:
        cid = _capture_id(stream.cuda_stream)
        if cid is not None:
            key = key + (cid,)
            buf = _counters.get(key)
        if buf is None:
            buf = torch.zeros(N_COUNTERS, dtype=torch.int32, device=dev)
            _counters[key] = buf
    return buf


def call(name, *args):
    fn = getattr(lib(), name)
    timer = KernelTimer.active
    rc = timer.record(name, lambda: fn(*args)) if timer else fn(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with code {rc}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("tgfr kernels take device tensors only (no CPU path)")
    return t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream
