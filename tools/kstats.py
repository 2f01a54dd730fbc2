"""Short table of a rocprofv3 kernel_stats.csv: calls, average and total microseconds per kernel."""
import csv
import re
import sys

for path in sys.argv[1:]:
    print(path)
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Name"].replace("void ", "").replace("protoseg::(anonymous namespace)::", "")
            name = re.sub(r"\(.*", "", name)
            print(f"  {name[:70]:70s} {int(row['Calls']):6d} {float(row['AverageNs']) / 1e3:9.2f} us "
                  f"{float(row['TotalDurationNs']) / 1e3:10.1f} us total")
