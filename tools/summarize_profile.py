"""Summarise a rocprofv3 round directory into profiles/rNN/summary.md and
profiles/rNN/pmc.json: per-kernel stats (trace pass) and per-kernel HBM bytes
from the FETCH_SIZE and WRITE_SIZE passes (FETCH_SIZE doubled: on gfx950 it
reports half the bytes of wide coalesced streaming reads, MI355X_MICROARCH.md
'HBM').

pmc.json is keyed by bench configuration (bench.config_key), so bench.py only
ever attaches traffic measured on its own configuration:
  {"configs": {"b64_w32_bf16_n1": {"source": ..., "kernels": {name: {...}}}}}
where name is either a kernel's short name or a C-ABI entry point whose
launches are the sum of its kernels (ABI_KERNELS).

Usage: python tools/summarize_profile.py <gpurun_out/prof_rNN> <profiles/rNN> <config_key>
"""
import collections
import csv
import json
import os
import sys

# ABI entry point -> alternative kernel sets (the first set fully present wins);
# one ABI call launches every kernel of its set once
ABI_KERNELS = {"tgfr_wr_bwd": (("wr_bwd_duo_kernel", "wr_reduce_frag_kernel"),
                               ("wr_bwd_duo_kernel",),
                               ("wr_bwd_pipe_kernel", "wr_reduce_frag_kernel"),
                               ("wr_bwd_wide2_kernel", "wr_reduce_frag_kernel"),
                               ("wr_bwd_wide2_kernel",),
                               ("wr_bwd_pipe_kernel", "wr_reduce_kernel"),
                               ("wr_bwd_wide_kernel", "wr_reduce_kernel"),
                               ("wr_bwd_kernel", "wr_reduce_kernel")),
               "tgfr_wr_fwd": (("wr_fwd_duo_kernel",), ("wr_fwd_pipe_kernel",),
                               ("wr_fwd_res2_kernel",),
                               ("wr_fwd_res_kernel",),
                               ("wr_fwd_kernel",))}


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0]


def base(name):
    return short(name).split("<")[0]


def read_pmc(path):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def entry_timings(trace_csv, names, steps):
    """Per-call durations of a C-ABI entry whose launches are the kernels
    `names` (base names, one launch each per call) from the kernel trace:
    (isolated, in_step) averages in us.  isolated = the longest run of
    back-to-back calls with nothing else dispatched between them (bench.py's
    HIP-event re-launch burst, _hip.KernelTimer); in_step = the last `steps`
    calls (the timed graph replays, beside the other stream's kernels).  A
    call's duration = first kernel's start .. last kernel's end."""
    rows = list(csv.DictReader(open(trace_csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    calls, i, seq = [], 0, list(names)
    while i < len(rows):
        if base(rows[i]["Kernel_Name"]) == seq[0] and i + len(seq) <= len(rows) and all(
                base(rows[i + j]["Kernel_Name"]) == seq[j] for j in range(len(seq))):
            calls.append((i, int(rows[i]["Start_Timestamp"]),
                          int(rows[i + len(seq) - 1]["End_Timestamp"])))
            i += len(seq)
        else:
            i += 1
    if not calls:
        return None, None
    runs, cur = [], [calls[0]]
    for c in calls[1:]:
        if c[0] == cur[-1][0] + len(seq):
            cur.append(c)
        else:
            runs.append(cur)
            cur = [c]
    runs.append(cur)
    burst = max(runs, key=len)
    avg = lambda cs: sum(e - s for _, s, e in cs) / len(cs) / 1e3  # noqa: E731
    return round(avg(burst), 2), round(avg(calls[-steps:]), 2)


def main(src, dst, key, steps=20):
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "bench_kernel_stats.csv"))))
    fetch = read_pmc(os.path.join(src, "fetch", "bench_counter_collection.csv"))
    write = read_pmc(os.path.join(src, "write", "bench_counter_collection.csv"))
    lines = ["# rocprofv3 summary", "", f"Configuration `{key}`. Trace: `rocprofv3 "
             "--kernel-trace --stats -- python3 bench.py ... --no-cpu --alt-precision ''` "
             "(graph replay). HBM bytes: separate `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` "
             "passes over eager launches; read = 2 x FETCH_SIZE (gfx950 correction).", "",
             "| kernel | calls | avg us | total % | read MB | write MB |",
             "|---|---|---|---|---|---|"]
    kernels = {}
    for r in stats:
        k = short(r["Name"])
        f, w = fetch.get(k), write.get(k)
        rd = None if f is None else 2 * f * 1024
        wr = None if w is None else w * 1024
        avg_us = float(r["AverageNs"]) / 1e3
        kernels[k] = {"avg_us": round(avg_us, 2), "calls": int(r["Calls"]),
                      "read_bytes": None if rd is None else int(rd),
                      "write_bytes": None if wr is None else int(wr),
                      "hbm_bytes_per_launch": None if rd is None or wr is None
                      else int(rd + wr)}
        if len(lines) < 40:
            fmt = lambda v: "-" if v is None else f"{v / 1e6:.1f}"  # noqa: E731
            lines.append(f"| `{k[:80]}` | {r['Calls']} | {avg_us:.1f} | "
                         f"{float(r['Percentage']):.1f} | {fmt(rd)} | {fmt(wr)} |")
    by_base = collections.defaultdict(list)
    for k in kernels:
        by_base[base(k)].append(k)
    abi_lines = ["", "C-ABI entry points (sum of their kernels' averages per call; and per "
                 "call from the trace: the isolated back-to-back re-launch burst bench.py times "
                 "with HIP events, and the last 20 graph-replayed steps):", "",
                 "| entry | kernels | avg us | isolated us | in-step us | HBM MB per call |",
                 "|---|---|---|---|---|---|"]
    for abi, sets in ABI_KERNELS.items():
        for names in sets:
            if all(n in by_base for n in names):
                ks = [max(by_base[n], key=lambda k: kernels[k]["calls"]) for n in names]
                us = sum(kernels[k]["avg_us"] for k in ks)
                hbm = [kernels[k]["hbm_bytes_per_launch"] for k in ks]
                tot = None if None in hbm else sum(hbm)
                iso, step = entry_timings(os.path.join(src, "trace", "bench_kernel_trace.csv"),
                                          names, steps)
                kernels[abi] = {"kernels": ks, "avg_us": round(us, 2),
                                "avg_us_isolated": iso, "avg_us_in_step": step,
                                "hbm_bytes_per_launch": tot}
                abi_lines.append(f"| `{abi}` | {' + '.join(base(k) for k in ks)} | {us:.1f} | "
                                 f"{iso} | {step} | "
                                 f"{'-' if tot is None else f'{tot / 1e6:.1f}'} |")
                break
    lines += abi_lines
    os.makedirs(dst, exist_ok=True)
    out_path = os.path.join(dst, "pmc.json")
    data = json.load(open(out_path)) if os.path.exists(out_path) else {"configs": {}}
    data.setdefault("configs", {})[key] = {
        "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; "
                  "hbm_bytes_per_launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024",
        "kernels": kernels}
    json.dump(data, open(out_path, "w"), indent=1)
    md = os.path.join(dst, f"summary_{key}.md")
    open(md, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
