"""Print a rocprofv3 kernel_stats.csv as name / calls / avg us / total %."""
import csv
import sys

for path in sys.argv[1:]:
    print("==", path)
    for r in csv.DictReader(open(path)):
        print(f'{r["Name"][:70]:70s} calls={r["Calls"]:>4} avg_us={float(r["AverageNs"])/1e3:10.1f} pct={float(r["Percentage"]):5.1f}')
