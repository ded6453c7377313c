"""Benchmark: face-caption pairs/s of the TGFR stage-1 train step (hot path).

    python bench.py [--gpus N --steps K --warmup W --precision bf16|fp32]

For N > 1 the driver launches one process per GPU with torch.distributed.run
(RCCL over xGMI); rank r owns images [r*B, (r+1)*B) and all-gathers the text
side, so each rank's contrastive losses see the whole global batch
(weak scaling: B = 64 images per GPU).

A step is one pass of the hot path over one batch of synthetic frozen-encoder
outputs already resident in HBM (BASELINE.json configs[1]: iResNet-100
features and BERT-base last hidden states, bs = 64/GPU, 32-token captions ->
30 words): the frozen text head (TextHeading, under no_grad as in
utils/dataset_utils.py:38-46), the image head (IMIM self-attention),
words_loss, sent_loss, global_loss, the two ArcMargin/focal identity losses,
backward, and both optimiser steps (src/train_encoders_bert.py:254-331).  The
frozen backbones (iResNet-100, BERT) run under torch.no_grad in the reference
and are not part of the measured step.

Output: ONE JSON line on rank 0 with the driver's fields plus
  roofline      dominant HIP kernel: algorithmic FLOPs per launch / its average
                duration (HIP events on the launch stream, second timed pass)
  cpu_baseline  the CPU oracle (oracle/tgfr_oracle.py) timed on the host cores
                for a bounded number of steps of the same workload (rank 0, N=1)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

R, D = 196, 256
PEAK_BF16_TFLOPS = 2500.0     # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=64, help="images per GPU")
    p.add_argument("--words", type=int, default=32, help="bert_words_num (T = words-2)")
    p.add_argument("--precision", default="bf16", choices=["bf16", "fp32", "fp16"])
    p.add_argument("--alt-precision", default="fp16,fp32",
                   help="also time these precision modes (comma list, '' to skip)")
    p.add_argument("--cpu-steps", type=int, default=6)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-text-head", action="store_true",
                   help="start from ready-made word / sentence features (the round-2 "
                        "workload) instead of running TextHeading in the step")
    p.add_argument("--eager", action="store_true",
                   help="launch kernels one by one instead of replaying a HIP graph")
    p.add_argument("--simulate-world", type=int, default=0,
                   help="one process plays rank 0 of N replicas (dist.ReplicaGroup): the "
                        "per-GPU work of an N-GPU step, no inter-GPU traffic; prints a "
                        "projection line, not the driver's metric line")
    return p.parse_args()


def sync_barrier(ctx):
    torch.cuda.synchronize()
    if ctx.multiprocess:
        dist.barrier()
    torch.cuda.synchronize()


def run_steps(trainer, batch, n):
    out = None
    for _ in range(n):
        out = trainer.step(batch)
    return out


def time_steps(trainer, batch, ctx, steps, warmup):
    run_steps(trainer, batch, warmup)
    sync_barrier(ctx)
    t0 = time.perf_counter()
    out = run_steps(trainer, batch, steps)
    sync_barrier(ctx)
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
    if ctx.multiprocess:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item(), out


def kernel_profile(trainer, batch, steps):
    """Per-ABI-call HIP-event timings over eager steps, plus back-to-back
    replays of the word<->region kernels' first calls; returns (summary, timer)."""
    from text_guided_face_recognition_amd._hip import KernelTimer
    with KernelTimer(replay=("tgfr_wr_fwd", "tgfr_wr_bwd")) as kt:
        run_steps(trainer, batch, steps)
    return kt.summary(), kt


def config_key(args, world):
    """The bench configuration a PMC measurement belongs to."""
    return f"b{args.batch}_w{args.words}_{args.precision}_n{world}"


def committed_entry(kernel, key):
    """The newest round's committed profile entry (profiles/rNN/pmc.json,
    tools/summarize_profile.py) of `kernel` for THIS configuration, or {}."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                          "profiles", "r*", "pmc.json")))
    for f in reversed(files):
        entry = json.load(open(f)).get("configs", {}).get(key, {}).get("kernels", {}).get(kernel)
        if entry is not None:
            return entry
    return {}


def pmc_traffic(kernel, key):
    """HBM bytes per launch of `kernel` measured for THIS configuration `key`
    (config_key) by the newest round's committed PMC passes
    (profiles/rNN/pmc.json, tools/summarize_profile.py: separate FETCH_SIZE /
    WRITE_SIZE rocprofv3 passes, FETCH_SIZE doubled per MI355X_MICROARCH.md
    'HBM').  None when no round measured this configuration: a number from
    another configuration is never attached."""
    import glob
    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                          "profiles", "r*", "pmc.json")))
    for f in reversed(files):
        data = json.load(open(f))
        entry = data.get("configs", {}).get(key, {}).get("kernels", {}).get(kernel)
        if entry is not None:
            return entry.get("hbm_bytes_per_launch")
    return None


def rocprof_fracs(flop, entry):
    """Peak fractions of a word<->region entry from its committed rocprof
    durations (isolated re-launch burst, in-step graph replay)."""
    out = {}
    for k in ("isolated", "in_step"):
        us = entry.get(f"avg_us_{k}")
        out[f"frac_rocprof_{k}"] = None if not us else round(
            flop / (us * 1e-6) / 1e12 / PEAK_BF16_TFLOPS, 4)
    return out


def host_cores():
    """(cores this process may run on, the machine's CPU count): the CPU
    affinity mask, capped by a cgroup CPU quota when one is set."""
    total = os.cpu_count() or 1
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = total
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            avail = max(1, min(avail, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return avail, total


def cpu_baseline(args, n_words):
    """The CPU oracle restatement of the same step on the host cores."""
    from oracle import tgfr_oracle as O
    threads, machine = host_cores()
    torch.set_num_threads(threads)
    b = args.batch
    gen = torch.Generator().manual_seed(100)
    unit = lambda x: x / x.norm(dim=-1, keepdim=True)  # noqa: E731
    g = torch.randn(b, 512, generator=gen)
    local = torch.randn(b, 256, 14, 14, generator=gen)
    words = unit(torch.randn(b, n_words, 256, generator=gen)).transpose(1, 2)
    sent = unit(torch.randn(b, 256, generator=gen))
    cls = torch.randint(0, 10000, (b,), generator=gen)
    hidden = torch.randn(b, n_words + 1, 768, generator=gen)
    conv_w, conv_b = [], []
    for k in (2, 3, 4):                      # Bert_Word_Mapping, models/models.py:177-179
        conv = torch.nn.Conv2d(1, 256, (k, 768))
        conv_w.append(conv.weight.detach())
        conv_b.append(conv.bias.detach())
    text_head = not args.no_text_head
    p = {}

    def lin(o, i):
        w = torch.empty(o, i)
        torch.nn.init.kaiming_uniform_(w, a=5 ** 0.5)
        return w.requires_grad_(), torch.zeros(o).requires_grad_()
    p["q_w"], p["q_b"] = lin(256, 256)
    p["k_w"], p["k_b"] = lin(256, 256)
    p["v_w"], p["v_b"] = lin(256, 256)
    for k in ("q_w", "k_w", "v_w"):
        p[k] = p[k].detach().reshape(256, 256, 1, 1).requires_grad_()
    hp = {"sa_" + k: v for k, v in p.items()}
    hp["bn_w"], hp["bn_b"] = torch.ones(256).requires_grad_(), torch.zeros(256).requires_grad_()
    hp["ln_w"] = torch.ones(256, 14, 14).requires_grad_()
    hp["ln_b"] = torch.zeros(256, 14, 14).requires_grad_()
    w1, hp["c1_b"] = lin(128, 256)
    w2, hp["c2_b"] = lin(256, 128)
    hp["c1_w"] = w1.detach().reshape(128, 256, 1, 1).requires_grad_()
    hp["c2_w"] = w2.detach().reshape(256, 128, 1, 1).requires_grad_()
    hp["pl_w"], hp["pl_b"] = lin(256, 256)
    hp["pg_w"], hp["pg_b"] = lin(256, 512)
    arc_i = torch.empty(4500, 256)
    torch.nn.init.xavier_uniform_(arc_i)
    arc_t = arc_i.clone()
    arc_i.requires_grad_()
    arc_t.requires_grad_()
    opt_h = torch.optim.Adam(list(hp.values()), lr=1e-3, betas=(0.5, 0.999))
    opt_c = torch.optim.SGD([arc_i, arc_t], lr=0.1, momentum=0.9, weight_decay=5e-5)
    labels = torch.arange(b)
    cls_np = cls.numpy()
    cls_ids = cls % 4500

    def step():
        w_, s_ = words, sent
        if text_head:
            with torch.no_grad():
                w_, s_ = O.text_heading(hidden, conv_w, conv_b, n_words + 2)
        gp, r = O.image_heading(g, local, hp)
        opt_h.zero_grad()
        opt_c.zero_grad()
        w0, w1_, _, _ = O.words_loss(r, w_, labels, None, n_words, 4.0, 5.0, 10.0)
        s0, s1, _ = O.sent_loss(gp, s_, labels, cls_np, 10.0)
        tid = O.focal_loss(O.arc_margin(s_, arc_t, cls_ids, s=35), cls_ids)
        iid = O.focal_loss(O.arc_margin(gp, arc_i, cls_ids, s=30), cls_ids)
        cl, _ = O.global_loss(gp, s_)
        total = w0 + w1_ + s0 + s1 + 100 * (tid + iid) + 2.0 * cl
        total.backward()
        opt_h.step()
        opt_c.step()

    step()                                   # warm-up
    times = []
    for _ in range(args.cpu_steps):
        t0 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t0)
    times.sort()
    med = times[len(times) // 2]
    return {"value": round(b / med, 3), "unit": "pairs/s", "cores": threads,
            "machine_cpus": machine, "kind": "port",
            "sample": f"{args.cpu_steps} steps (+1 warm-up) of the same bs={b}, T={n_words} "
                      f"stage-1 step{' (TextHeading included)' if text_head else ''} "
                      f"through the fp32 oracle on {threads} torch threads "
                      f"(every core this process may use; the machine has {machine}); "
                      f"median step {med * 1000:.0f} ms"}


def spawn_ranks(args):
    """`bench.py --gpus N` run directly (no WORLD_SIZE): start N ranks with
    torch.distributed.run as a CHILD process (nothing here has touched the
    GPU) and exit with its status."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    from text_guided_face_recognition_amd.config import make_args
    from text_guided_face_recognition_amd.dist import DistContext, ReplicaGroup, init_from_env
    from text_guided_face_recognition_amd.train import GraphedStep, Train, synthetic_batch

    ctx = init_from_env()
    if args.gpus != ctx.world and args.simulate_world <= 1:
        raise SystemExit(f"--gpus {args.gpus} but {ctx.world} rank(s) were launched")
    if args.simulate_world > 1 and not ctx.active:
        ctx = DistContext(ReplicaGroup(args.simulate_world))
        args.no_cpu = True
    local_rank = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    n_words = args.words - 2

    def build(precision):
        torch.manual_seed(100)
        targs = make_args(batch_size=args.batch, bert_words_num=args.words,
                          num_classes=4500, precision=precision)
        return Train(targs, dev, ctx)

    batch = synthetic_batch(args.batch, n_words, dev, seed=100 + 1000 * ctx.rank,
                            bert_hidden=not args.no_text_head)
    batch = batch[:-1] + (batch[-1] % 4500,)

    use_graph = not args.eager

    def runner(tr):
        return GraphedStep(tr, batch) if use_graph else tr

    trainer = build(args.precision)
    prof, ktimer = kernel_profile(trainer, batch, max(3, min(args.steps, 10)))
    elapsed, out = time_steps(runner(trainer), batch, ctx, args.steps, args.warmup)
    n = ctx.world
    pairs = n * args.batch * args.steps
    value = pairs / elapsed

    # the other precision modes of the same step: fp16 (the word<->region
    # contraction on fp16 operands, which meets the north star's 1e-3 on
    # logits) and fp32 (split-bf16 operands, the parity mode)
    alt = {}
    for ap in [a for a in args.alt_precision.split(",") if a and a != args.precision]:
        tr2 = build(ap)
        prof2, kt2 = kernel_profile(tr2, batch, max(3, min(args.steps, 10)))
        e2, _ = time_steps(runner(tr2), batch, ctx, args.steps, args.warmup)
        alt[ap] = {"value": round(pairs / e2, 2), "ms_per_step": round(e2 / args.steps * 1000, 4),
                   "vs_headline_step": round(elapsed / e2, 4),
                   "replayed_ms": {k: round(v, 4) for k, v in kt2.replayed.items()},
                   "eager_entry_ms": {k: round(v[1], 4) for k, v in prof2.items()}}
        del tr2
    alt = alt or None

    if isinstance(ctx.group, ReplicaGroup):
        print(json.dumps({
            "simulated_world": n, "projected_value": round(value, 2), "unit": "pairs/s",
            "ms_per_step": round(elapsed / args.steps * 1000, 4),
            "note": "one GPU doing rank 0's share of an N-GPU step (B_l images x B_l*N "
                    "captions); collectives replaced by local copies",
            "eager_entry_ms": {k: round(v[1], 4) for k, v in sorted(prof.items())}}), flush=True)
        return
    if ctx.rank != 0:
        if ctx.multiprocess:
            dist.barrier()
        return

    # roofline of the dominant word<->region kernel (SURVEY.md 8(d):
    # fwd 4*R*D*T and bwd 6*R*D*T FLOPs per (image, caption) pair)
    pair_count = args.batch * args.batch * n
    flops = {"tgfr_wr_fwd": 4 * R * D * n_words * pair_count,
             "tgfr_wr_bwd": 6 * R * D * n_words * pair_count}
    # the dominant word<->region entry point by its replayed launch time
    dominant = max((k for k in ktimer.replayed if k in flops), key=lambda k: ktimer.replayed[k])
    # the dominant kernel's launch duration: HIP events around 20 back-to-back
    # re-launches with the step's own arguments (inside the step, while its
    # buffers are alive), on the stream it runs on
    dom_ms = ktimer.replayed[dominant]
    achieved = flops[dominant] / (dom_ms * 1e-3) / 1e12
    roofline = {"bound": "mfma", "kernel": dominant, "achieved": round(achieved, 2),
                "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                "traffic": pmc_traffic(dominant, config_key(args, n)),
                "avg_launch_ms": round(dom_ms, 4),
                "flop_per_launch": flops[dominant],
                "timing": "HIP events around 20 back-to-back re-launches of the call "
                          "(the isolated-launch figure); frac_rocprof_* from the committed "
                          "rocprof trace of this configuration (profiles/rNN/pmc.json): the "
                          "same burst, and the graph-replayed step beside the side stream",
                **rocprof_fracs(flops[dominant], committed_entry(dominant, config_key(args, n))),
                # the other word<->region entry point, timed the same way
                "others": {k: {"avg_launch_ms": round(v, 4),
                               "achieved": round(flops[k] / (v * 1e-3) / 1e12, 2),
                               "frac": round(flops[k] / (v * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4),
                               **rocprof_fracs(flops[k], committed_entry(k, config_key(args, n))),
                               "traffic": pmc_traffic(k, config_key(args, n))}
                           for k, v in ktimer.replayed.items() if k in flops and k != dominant}}

    cpu = None
    if not args.no_cpu and n == 1:
        cpu = cpu_baseline(args, n_words)

    line = {
        "metric": "face-caption pairs/sec train step (iResNet100+BERT, bs=64/GPU) "
                  "at 1/2/4/8 MI355X",
        "value": round(value, 2), "unit": "pairs/s", "n_gpus": n, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1000, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": args.precision, "data": "synthetic",
        "config": {"workload": ("FCAM stage-1 train step (BASELINE configs[1]): " +
                                ("" if args.no_text_head else "frozen TextHeading + ") +
                                "IMIM head + words/sent/global losses + identity heads + "
                                "backward + optimiser, on iResNet-100 / BERT-base-shaped "
                                "frozen-backbone outputs"),
                   "global_batch": args.batch * n, "seq_len": args.words,
                   "words_per_caption": n_words, "parallelism": f"dp{n}",
                   "launch": "hip-graph" if use_graph else "eager",
                   # one process: TextHeading and the g' branch on a side stream
                   # beside IMIM and the word<->region branch (train.Train.step)
                   "streams": 2 if getattr(trainer, "_side", None) is not None else 1},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "eager_entry_ms": {k: round(v[1], 4) for k, v in sorted(prof.items())},
        "alt_precision": alt,
    }
    print(json.dumps(line), flush=True)
    if ctx.multiprocess:
        dist.barrier()


if __name__ == "__main__":
    main()
