"""Summarise a rocprofv3 round directory into profiles/rNN/summary.md:
per-kernel stats (trace pass) and per-kernel HBM bytes from the FETCH_SIZE and
WRITE_SIZE passes (FETCH_SIZE doubled: on gfx950 it reports half the bytes of
wide coalesced streaming reads, MI355X_MICROARCH.md 'HBM')."""
import collections
import csv
import os
import sys


def main(src, dst):
    stats = list(csv.DictReader(open(os.path.join(src, "trace", "bench_kernel_stats.csv"))))
    lines = ["# rocprofv3 summary", "", "Command: `rocprofv3 --kernel-trace --stats -- "
             "python3 bench.py --steps 20 --warmup 5 --no-cpu --alt-precision ''` "
             "(graph replay, bf16 mode, B=64, T=30).", "",
             "| kernel | calls | avg us | total % |", "|---|---|---|---|"]
    for r in stats[:25]:
        name = r["Name"].split("(")[0].replace("void ", "")[:70]
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
            for tag in ("wr_fwd_kernel", "wr_bwd_kernel", "wr_reduce_kernel", "prep_rows_kernel"):
                if tag in r["Kernel_Name"]:
                    acc[tag].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            pmc[k][name] = sum(v) / len(v)
    for k, v in pmc.items():
        f, w = v.get("fetch", 0.0), v.get("write", 0.0)
        lines.append(f"| `{k}` | {f:.0f} | {2 * f / 1024:.1f} | {w / 1024:.1f} |")
    os.makedirs(dst, exist_ok=True)
    open(os.path.join(dst, "summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
