"""Summarise a rocprofv3 round directory into profiles/rNN/summary.md:
per-kernel stats (trace pass) and per-kernel HBM bytes from the FETCH_SIZE and
WRITE_SIZE passes (FETCH_SIZE doubled: on gfx950 it reports half the bytes of
wide coalesced streaming reads, MI355X_MICROARCH.md 'HBM')."""
import collections
import csv
import json
import os
import sys

# ABI entry point -> kernel name(s) in the trace
ABI_KERNELS = {"tgfr_wr_bwd": ("wr_bwd_pipe_kernel", "wr_bwd_kernel"),
               "tgfr_wr_fwd": ("wr_fwd_pipe_kernel", "wr_fwd_res_kernel", "wr_fwd_kernel")}


def main(src, dst):
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "bench_kernel_stats.csv"))))
    lines = ["# rocprofv3 summary", "", "Command: `rocprofv3 --kernel-trace --stats -- "
             "python3 bench.py --steps 20 --warmup 5 --no-cpu --alt-precision ''` "
             "(graph replay, bf16 mode, B=64, T=30).", "",
             "| kernel | calls | avg us | total % |", "|---|---|---|---|"]
    for r in stats[:25]:
        name = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        name = name.split("(")[0][:70]
        lines.append(f"| `{name}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{float(r['Percentage']):.1f} |")
    lines += ["", "HBM traffic per launch (separate --pmc passes, eager launches):", "",
              "| kernel | FETCH_SIZE KB (raw) | read MB (x2 corrected) | WRITE_SIZE MB |",
              "|---|---|---|---|"]
    pmc = collections.defaultdict(dict)
    for name in ("fetch", "write"):
        rows = csv.DictReader(open(os.path.join(src, name, "bench_counter_collection.csv")))
        acc = collections.defaultdict(list)
        for r in rows:
            for tag in ("wr_fwd_pipe_kernel", "wr_bwd_pipe_kernel", "wr_fwd_res_kernel",
                        "wr_fwd_kernel", "wr_bwd_kernel", "wr_reduce_kernel", "prep_rows_kernel"):
                if tag in r["Kernel_Name"]:
                    acc[tag].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            pmc[k][name] = sum(v) / len(v)
    for k, v in pmc.items():
        f, w = v.get("fetch", 0.0), v.get("write", 0.0)
        lines.append(f"| `{k}` | {f:.0f} | {2 * f / 1024:.1f} | {w / 1024:.1f} |")
    os.makedirs(dst, exist_ok=True)
    # bytes per launch for bench.py's roofline.traffic (FETCH_SIZE / WRITE_SIZE
    # are KB; FETCH_SIZE doubled for gfx950)
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, "
                     "bench.py --eager bf16 B=64 T=30", "kernels": {}}
    for abi, names in ABI_KERNELS.items():
        for n in names:
            if n in pmc:
                f, w = pmc[n].get("fetch", 0.0), pmc[n].get("write", 0.0)
                out["kernels"][abi] = {"kernel": n, "fetch_kb_raw": round(f, 1),
                                       "write_kb": round(w, 1),
                                       "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024)}
                break
    json.dump(out, open(os.path.join(dst, "pmc.json"), "w"), indent=1)
    open(os.path.join(dst, "summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
