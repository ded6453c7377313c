"""Average SQ counters per launch of the word<->region kernels from
rocprofv3 --pmc passes (tools/pmc_wr.sh) -> a JSON file under profiles/,
with the derived issue figures the roofline discussion uses.

    python tools/summarize_sq.py OUT.json CONFIG_NOTE gpurun_out/pmcw1 gpurun_out/pmcw2 ...
"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = ("wr_bwd_duo_kernel", "wr_fwd_duo_kernel", "wr_bwd_pipe_kernel", "wr_fwd_pipe_kernel",
           "wr_bwd_wide2_kernel", "wr_fwd_res2_kernel", "wr_reduce_frag_kernel")
# waves that share one SIMD for the kernel's whole life (its workgroup size / 256)
WAVES_PER_SIMD = {"wr_bwd_duo_kernel": 2, "wr_fwd_duo_kernel": 2}


def main(out, note, *dirs):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            per = collections.defaultdict(float)
            for row in csv.DictReader(open(f)):
                name = row["Kernel_Name"].replace("(anonymous namespace)::", "")
                k = next((k for k in KERNELS if k in name), None)
                if k is None:
                    continue
                per[(k, row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
            for (k, _, c), v in per.items():
                acc[k][c].append(v)
    res = {}
    for k, cs in acc.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        res[k] = avg
    flops = {"wr_bwd_pipe_kernel": 6 * 196 * 256 * 30 * 64 * 64,
             "wr_bwd_duo_kernel": 6 * 196 * 256 * 30 * 64 * 64,
             "wr_fwd_duo_kernel": 4 * 196 * 256 * 30 * 64 * 64,
             "wr_fwd_pipe_kernel": 4 * 196 * 256 * 30 * 64 * 64}
    derived = {}
    for k, avg in res.items():
        d = {}
        if avg.get("SQ_INSTS_MFMA", 0) <= 0:
            derived[k] = d
            continue
        if k in flops:
            d["issued_mfma_flop_over_algorithmic"] = avg["SQ_INSTS_MFMA"] * 32768 / flops[k]
        if "SQ_INSTS_VALU" in avg:
            # (SQ_INSTS_VALU counts the MFMAs too)
            d["valu_insts_per_mfma"] = (avg["SQ_INSTS_VALU"] - avg["SQ_INSTS_MFMA"]) / avg["SQ_INSTS_MFMA"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in avg and "SQ_WAVE_CYCLES" in avg:
            # the matrix core's busy cycles (32 per 32x32x16 MFMA) over the
            # SIMDs' resident cycles: the waves' (quad-cycles x 4) divided by
            # the waves that share a SIMD (co-resident for the whole kernel)
            w = WAVES_PER_SIMD.get(k, 1)
            d["mfma_busy_over_simd_cycles"] = avg["SQ_VALU_MFMA_BUSY_CYCLES"] / (
                4 * avg["SQ_WAVE_CYCLES"] / w)
        if "SQ_WAIT_ANY" in avg and "SQ_WAVE_CYCLES" in avg:
            d["wait_any_over_wave_cycles"] = avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"]
        derived[k] = d
    json.dump({"config": note, "source": "rocprofv3 --pmc SQ passes (tools/pmc_wr.sh), "
               "averages per launch; *_CYCLES of SQ_WAVE / SQ_WAIT / SQ_BUSY in quad-cycles",
               "kernels": res, "derived": derived}, open(out, "w"), indent=1)
    print(json.dumps(derived, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
