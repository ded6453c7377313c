"""Timeline of one graph-replayed train step from a rocprofv3 kernel trace:
each kernel's start / end offset from the step's first kernel, its queue
(stream), and the main-stream gaps -- what is on the critical path.

    python tools/timeline.py <bench_kernel_trace.csv> [--step K]

K indexes the word-region forward launches (one per step); default -3.
"""
import csv
import re
import sys


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    m = re.match(r"([\w:<>, ]+?)\(", n)
    return (m.group(1) if m else n)[:48]


def main(path, which=-3):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "wr_fwd" in r["Kernel_Name"]]
    # a step = from the first kernel after the previous step's last optimiser
    # launch; approximate: the window between two wr_fwd launches, shifted back
    # to the step's first kernel (the IMIM BN statistics)
    lo = idx[which]
    while lo > 0 and not any(k in rows[lo]["Kernel_Name"] for k in ("bn_stats", "imim_prep")):
        lo -= 1
    hi = idx[which + 1]
    while hi > 0 and not any(k in rows[hi]["Kernel_Name"] for k in ("bn_stats", "imim_prep")):
        hi -= 1
    step = rows[lo:hi]
    t0 = int(step[0]["Start_Timestamp"])
    t_end = max(int(r["End_Timestamp"]) for r in step)
    queues = sorted({r["Queue_Id"] for r in step}, key=lambda q: -sum(
        1 for r in step if r["Queue_Id"] == q))
    last_end = {}
    print(f"{'start':>7} {'end':>7} {'dur':>6} {'gap':>6} q  kernel")
    for r in step:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        q = queues.index(r["Queue_Id"])
        gap = s - last_end.get(q, s)
        last_end[q] = e
        print(f"{s / 1e3:7.1f} {e / 1e3:7.1f} {(e - s) / 1e3:6.1f} {gap / 1e3:6.1f} {q}  "
              f"{short(r['Kernel_Name'])} grid={r['Grid_Size_X']}")
    print(f"step span {(t_end - t0) / 1e3:.1f} us, next step starts at "
          f"{(int(rows[hi]['Start_Timestamp']) - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    k = sys.argv.index("--step") if "--step" in sys.argv else None
    main(sys.argv[1], int(sys.argv[k + 1]) if k else -3)
