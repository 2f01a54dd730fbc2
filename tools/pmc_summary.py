"""Summarise rocprofv3 --pmc passes (tools/pmc_sq.sh output): mean counter value per kernel."""
import collections
import csv
import glob
import os
import sys


def main(root):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in sorted(glob.glob(os.path.join(root, "p*", "*_counter_collection.csv"))):
        per, names = collections.defaultdict(float), {}
        for r in csv.DictReader(open(path)):
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (d, c), v in per.items():
            agg[names[d].split("namespace)::")[-1][:40]][c].append(v)
    ks = [k for k in agg if "rocclr" not in k]
    cs = sorted({c for k in ks for c in agg[k]})
    print(f"{'':28s}" + "".join(f"{k[:22]:>24s}" for k in ks))
    for c in cs:
        print(f"{c:28s}" + "".join(f"{sum(agg[k][c]) / max(1, len(agg[k][c])):24.4g}" for k in ks))
    print("derived (per wave, cycles = 4 x quad-cycles):")
    for k in ks:
        a = {c: sum(v) / len(v) for c, v in agg[k].items()}
        w = a.get("SQ_WAVES", 0) or 1
        line = [f"wave_cyc {4 * a.get('SQ_WAVE_CYCLES', 0) / w:9.0f}"]
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if c in a and a.get("SQ_WAVE_CYCLES"):
                line.append(f"{c[3:]} {a[c] / a['SQ_WAVE_CYCLES']:.2f}")
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
            if c in a:
                line.append(f"{c[8:]}/w {a[c] / w:.0f}")
        print(f"  {k[:30]:30s} " + "  ".join(line))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_sq")
