"""Mean per-dispatch PMC counters of hb_eval_* per variant (gpurun_out/pmcab)."""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
res = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    tag = os.path.relpath(f, root).split(os.sep)[0].rsplit("_", 1)[0]
    for r in csv.DictReader(open(f)):
        if "hb_eval" in r["Kernel_Name"]:
            res[tag][r["Counter_Name"]].append(float(r["Counter_Value"]))
for tag in sorted(res):
    d = res[tag]
    print(tag, " ".join(f"{k}={sum(v)/len(v):.4g}" for k, v in sorted(d.items())))
