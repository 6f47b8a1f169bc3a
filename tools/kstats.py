"""Print the per-kernel average duration from a rocprofv3 --stats output dir."""
import csv
import glob
import sys

for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{float(r['AverageNs']) / 1e3:9.2f} us  x{r['Calls']:>5}  {r['Name'][:110]}")
