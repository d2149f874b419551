"""Summarise rocprofv3 PMC passes for the render kernel into JSON (dev tool).

Usage: pmc_summary.py OUT.json DIR [DIR ...]  (each DIR holds one
--pmc pass: *_counter_collection.csv). Per-dispatch values of the render
kernel are averaged over dispatches. HBM bytes follow MI355X_MICROARCH.md
§HBM: FETCH_SIZE (KiB) reads half the bytes of a wide coalesced stream on
gfx950, so hbm_read = 2 * FETCH_SIZE * 1024 is an upper estimate; WRITE_SIZE
(KiB) is exact for 16-B stores.
"""
import csv, glob, json, sys, collections

out, dirs = sys.argv[1], sys.argv[2:]
per = collections.defaultdict(list)
for d in dirs:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        byd = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if "render_kernel" not in r["Kernel_Name"]:
                continue
            byd[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        for disp, cs in byd.items():
            for k, v in cs.items():
                per[k].append(v)
avg = {k: sum(v) / len(v) for k, v in per.items()}
res = {"counters_per_dispatch": avg, "dispatches": {k: len(v) for k, v in per.items()}}
if "FETCH_SIZE" in avg or "WRITE_SIZE" in avg:
    fetch = avg.get("FETCH_SIZE", 0.0) * 1024
    write = avg.get("WRITE_SIZE", 0.0) * 1024
    res["hbm_read_bytes_raw"] = fetch
    res["hbm_read_bytes_corrected"] = 2 * fetch
    res["hbm_write_bytes"] = write
    res["hbm_bytes_per_launch"] = 2 * fetch + write
json.dump(res, open(out, "w"), indent=1, sort_keys=True)
print(json.dumps(res, indent=1, sort_keys=True))
