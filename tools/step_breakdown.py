"""Per-kernel breakdown of one graph-replayed train step from a rocprofv3
kernel trace (tools/profile_round.sh output).

    python tools/step_breakdown.py <bench_kernel_trace.csv> [--list] [--step K]

K indexes the word-region forward launches (one per step); default -3.
"""
import collections
import csv
import re
import sys


def main(path, listing=False, which=-3):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "wr_fwd" in r["Kernel_Name"]]
    step = rows[idx[which]:idx[which + 1]]
    t0, t1 = int(step[0]["Start_Timestamp"]), int(rows[idx[which + 1]]["Start_Timestamp"])
    fam = collections.defaultdict(lambda: [0, 0.0])
    for i, r in enumerate(step):
        n = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if listing:
            print(f"{i:3d} {d:7.1f} grid=({r['Grid_Size_X']},{r['Grid_Size_Y']},"
                  f"{r['Grid_Size_Z']}) wg={r['Workgroup_Size_X']} {n[:100]}")
        m = re.search(r"namespace\)::(\w+)", n)
        if m and not n.startswith("void at::"):
            k = "tgfr:" + m.group(1)
        elif "multi_tensor_apply" in n:
            k = "optimizer"
        elif "reduce_kernel" in n:
            k = "torch reduce"
        elif "elementwise" in n:
            k = "torch elementwise: " + ",".join(
                dict.fromkeys(re.findall(r"(\w+Functor\w*|direct_copy\w*)", n)))[:50]
        else:
            k = "other: " + n[:50]
        fam[k][0] += 1
        fam[k][1] += d
    tot = sum(v[1] for v in fam.values())
    print(f"kernels/step={len(step)} wall={(t1 - t0) / 1e3:.1f}us busy={tot:.1f}us")
    for k, v in sorted(fam.items(), key=lambda x: -x[1][1]):
        print(f"{v[0]:4d} {v[1]:8.1f}us {100 * v[1] / tot:5.1f}%  {k}")


if __name__ == "__main__":
    k = sys.argv.index("--step") if "--step" in sys.argv else None
    main(sys.argv[1], "--list" in sys.argv, int(sys.argv[k + 1]) if k else -3)
