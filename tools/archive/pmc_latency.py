"""Sum selected PMC counters per kernel over a rocprofv3 counter_collection.csv
(dev tool): python tools/archive/pmc_latency.py DIR [DIR ...] -> per kernel name
prefix, every counter's total and derived latencies (level / instructions)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(dirs):
    tot = defaultdict(lambda: defaultdict(float))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                key = name.split("(")[0].replace("void ", "").replace("rtamd::", "")
                tot[key][r["Counter_Name"]] += float(r["Counter_Value"])
    return tot


def main():
    tot = load(sys.argv[1:])
    for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", kv[1].get("SQ_INSTS_LDS", 0))):
        out = {n: round(v) for n, v in sorted(c.items())}
        if c.get("SQ_INSTS_LDS"):
            if c.get("SQ_INST_LEVEL_LDS"):
                out["lds_latency_cycles"] = round(c["SQ_INST_LEVEL_LDS"] / c["SQ_INSTS_LDS"], 1)
        if c.get("SQ_INSTS_VMEM") and c.get("SQ_INST_LEVEL_VMEM"):
            out["vmem_latency_cycles"] = round(c["SQ_INST_LEVEL_VMEM"] / c["SQ_INSTS_VMEM"], 1)
        if c.get("SQ_INSTS_SMEM") and c.get("SQ_INST_LEVEL_SMEM"):
            out["smem_latency_cycles"] = round(c["SQ_INST_LEVEL_SMEM"] / c["SQ_INSTS_SMEM"], 1)
        if c.get("SQ_LEVEL_WAVES") and c.get("SQ_BUSY_CYCLES"):
            out["avg_waves_resident"] = round(c["SQ_LEVEL_WAVES"] / c["SQ_BUSY_CYCLES"], 2)
        print(k, out)


if __name__ == "__main__":
    main()
