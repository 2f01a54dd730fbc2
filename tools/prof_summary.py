"""Summarise one tools/profile.sh run (rocprofv3 kernel-trace stats + separate FETCH_SIZE and
WRITE_SIZE passes) into a per-kernel JSON: calls, average duration, counters per dispatch and
the corrected HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md HBM
section: gfx950 FETCH_SIZE reports half of wide streaming reads; both counters are in KB).

usage: python tools/prof_summary.py gpurun_out/prof_<tag> profiles/<round>/prof_<tag>.json
"""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    name = name.split("(")[0]
    for pre in ("void ", "protoseg::(anonymous namespace)::"):
        name = name.replace(pre, "")
    return name.split("<")[0]


def counter_means(path):
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        per[r["Dispatch_Id"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
    agg = collections.defaultdict(list)
    for d, v in per.items():
        agg[names[d]].append(v)
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main(root, out):
    stats = {}
    for r in csv.DictReader(open(glob.glob(os.path.join(root, "trace", "*_kernel_stats.csv"))[0])):
        stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": round(float(r["AverageNs"]) / 1e3, 2),
                                   "min_us": round(float(r["MinNs"]) / 1e3, 2)}
    fetch = counter_means(glob.glob(os.path.join(root, "fetch", "*_counter_collection.csv"))[0])
    write = counter_means(glob.glob(os.path.join(root, "write", "*_counter_collection.csv"))[0])
    for k, s in stats.items():
        if k in fetch and k in write:
            s["FETCH_SIZE_KB"] = round(fetch[k], 1)
            s["WRITE_SIZE_KB"] = round(write[k], 1)
            s["hbm_bytes_per_launch"] = int(round((2 * fetch[k] + write[k]) * 1024))
    doc = {"source": root, "command": "tools/profile.sh: rocprofv3 --kernel-trace --stats | --pmc FETCH_SIZE | "
           "--pmc WRITE_SIZE (separate passes) over python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline",
           "kernels": dict(sorted(stats.items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["calls"]))}
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    for k, s in doc["kernels"].items():
        print(f"{k:34s} {s['calls']:5d} {s['avg_us']:9.2f} us  hbm/launch {s.get('hbm_bytes_per_launch', '-')}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
