"""Per-(kernel, grid) table of a rocprofv3 kernel_trace.csv: calls, average / min microseconds,
VGPRs and LDS. Splits a kernel launched at several shapes (the wide family's GEMM chain) into
its individual launches."""
import collections
import csv
import re
import sys

for path in sys.argv[1:]:
    print(path)
    groups = collections.OrderedDict()
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"].replace("void ", "").replace("protoseg::(anonymous namespace)::", "")
            name = re.sub(r"\(.*", "", name.replace("protoseg::", ""))
            grid = tuple(int(row[k]) // max(int(row[k.replace("Grid", "Workgroup")]), 1)
                         for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
            key = (name[:60], grid, row["VGPR_Count"], row["Accum_VGPR_Count"], row["LDS_Block_Size"])
            groups.setdefault(key, []).append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    for (name, grid, vg, ag, lds), ts in groups.items():
        ts.sort()
        print(f"  {name:60s} grid {str(grid):18s} v{vg}/a{ag} lds {lds:>6s} n={len(ts):4d} "
              f"med {ts[len(ts) // 2]:9.2f} min {ts[0]:9.2f} us")
