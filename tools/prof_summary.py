"""Summarise one tools/profile.sh run (per workload: rocprofv3 kernel-trace stats + separate
FETCH_SIZE and WRITE_SIZE passes) into per-kernel JSON: calls, average duration, counters per
dispatch and the corrected HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md
HBM section: gfx950 FETCH_SIZE reports half of wide streaming reads; both counters are in KB).
With --traffic, the per-launch HBM bytes are also merged into profiles/pmc_traffic.json under
the bench's config keys (what bench.py reports as roofline.traffic).

usage: python tools/prof_summary.py gpurun_out/prof_<tag> profiles/<round>/prof_<tag>.json [--traffic]
"""
import collections
import csv
import glob
import json
import os
import sys

# workload dir -> bench config key (bench.layer_report: B, C, map, P, K, x dtype, precision)
CONFIG_KEYS = {"p361": "B32_C64_65x65_P361_K19_f32_bf16x3", "p190": "B32_C64_65x65_P190_K19_f32_bf16x3",
               "rest": "B32_C64_65x65_P190_K19_f32_bf16x3"}
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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


def workload(root):
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
    return dict(sorted(stats.items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["calls"]))


def main(root, out, traffic):
    doc = {"source": root, "command": "tools/profile.sh: per workload, rocprofv3 --kernel-trace --stats | --pmc "
           "FETCH_SIZE | --pmc WRITE_SIZE (separate passes) over python3 bench.py --steps 20 --warmup 5 "
           "--no-cpu-baseline + the workload's flags", "workloads": {}}
    for wl in sorted(os.listdir(root)):
        if os.path.isdir(os.path.join(root, wl, "trace")):
            doc["workloads"][wl] = workload(os.path.join(root, wl))
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    for wl, ks in doc["workloads"].items():
        print(f"-- {wl}")
        for k, s in ks.items():
            print(f"{k:34s} {s['calls']:5d} {s['avg_us']:9.2f} us  hbm/launch {s.get('hbm_bytes_per_launch', '-')}")
    if traffic:
        path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        try:
            data = json.load(open(path))
        except (OSError, ValueError):
            data = {}
        data["_note"] = ("HBM bytes per launch = 2 x FETCH_SIZE (gfx950 reports half of wide streaming reads, "
                         f"MI355X_MICROARCH.md HBM section) + WRITE_SIZE, from {out} (tools/profile.sh + "
                         "tools/prof_summary.py)")
        # the layer workloads own their config's layer kernels; "rest" fills in the others
        for wl in sorted(doc["workloads"], key=lambda w: w == "rest", reverse=True):
            key = CONFIG_KEYS.get(wl)
            if key is None:
                continue
            for k, s in doc["workloads"][wl].items():
                if "hbm_bytes_per_launch" in s:
                    data.setdefault(key, {})[k] = {"hbm_bytes_per_launch": s["hbm_bytes_per_launch"],
                                                   "avg_us": s["avg_us"]}
        with open(path, "w") as f:
            json.dump(data, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], "--traffic" in sys.argv[3:])
