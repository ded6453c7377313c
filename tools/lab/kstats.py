"""Per-step kernel table from a rocprofv3 --stats csv (bench: 38 step replays)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1] + "/bench_kernel_stats.csv")))
per = float(sys.argv[2]) if len(sys.argv) > 2 else 38
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    n = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
    print(f"{n:62s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:8.1f} {float(r['TotalDurationNs'])/per/1e3:8.1f}")
print("total per step (us)", round(tot / per / 1e3, 1))
