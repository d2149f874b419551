"""Per-kernel counter totals of a tools/profile.sh output directory (dev tool).
Usage: pmc_peek.py DIR [kernel-substring]"""
import csv, glob, os, sys, collections
d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
tot = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if pat in k:
            tot[k.split("(")[0][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for f in glob.glob(os.path.join(d, "kt", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if pat in r["Name"]:
            print(f"{r['Name'][:90]:90s} calls {r['Calls']} avg_us {float(r['AverageNs'])/1e3:.1f}")
for k, c in tot.items():
    print(k)
    for n, v in sorted(c.items()):
        print(f"   {n:28s} {v:16.0f}")
