"""Summarise rocprofv3 counter CSVs (gpurun_out/pmcw1, pmcw2) per wr kernel:
per-dispatch averages, plus derived per-wave cycle shares."""
import collections
import csv
import sys

dirs = sys.argv[1:] or ["gpurun_out/pmcw1", "gpurun_out/pmcw2"]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in dirs:
    for r in csv.DictReader(open(f"{d}/w_counter_collection.csv")):
        k = r["Kernel_Name"]
        if "wr_" not in k:
            continue
        name = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, dd in agg.items():
    c = {n: sum(v) / len(v) for n, v in dd.items()}
    print(k, {n: round(v) for n, v in sorted(c.items())})
    w = c.get("SQ_WAVE_CYCLES")
    if w:
        print("   wait_any %.2f  wait_inst %.2f  active %.2f  (of wave cycles)" % (
            c.get("SQ_WAIT_ANY", 0) / w, c.get("SQ_WAIT_INST_ANY", 0) / w,
            c.get("SQ_ACTIVE_INST_ANY", 0) / w))
