"""Print per-kernel average durations (us) of rocprofv3 *_kernel_stats.csv files."""
import csv
import sys

for p in sys.argv[1:]:
    out = []
    for r in csv.DictReader(open(p)):
        out.append("%s=%.1f" % (r["Name"].split("(")[0].split("::")[-1].split("<")[0][:16], float(r["AverageNs"]) / 1000))
    print(p.split("/")[-2], " ".join(out))
