"""Timeline of catalog calls (BASELINE config C5) from a rocprofv3 kernel
trace: for each of the last calls, every launch's start offset from the
call's records launch, its duration, grid and stream, and the call's span
(records start -> last class end); then the per-kernel means over those calls.
Answers where a C5 call's 0.15 ms goes: the records launch, each size class,
the gaps between them, the serial tail.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c5tl -o c5 -- python bench.py --config C5 ...
    python scripts/c5_timeline.py gpurun_out/c5tl [--calls 20]
"""
import argparse
import csv
import glob
import json
import os
import re

import numpy as np

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--calls", type=int, default=20)
ap.add_argument("--json", default=None)
a = ap.parse_args()
f = sorted(glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True))[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))


def short(name):
    m = re.search(r"(hb_\w+|ds_\w+)(<[^()]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


# a call starts at each records (prep) launch
starts = [i for i, r in enumerate(rows) if "hb_prep_kernel" in r["Kernel_Name"]]
calls = []
for ci, si in enumerate(starts):
    end = starts[ci + 1] if ci + 1 < len(starts) else len(rows)
    calls.append(rows[si:end])
calls = calls[-a.calls - 1:-1]  # the last full calls (the kernel-timing pass)
per = {}
spans = []
for call in calls:
    t0 = int(call[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in call)
    spans.append((t1 - t0) / 1e3)
    for r in call:
        k = short(r["Kernel_Name"]) + f" grid={r.get('Grid_Size', r.get('Grid_Size_X', '?'))}"
        d = per.setdefault(k, {"start_us": [], "dur_us": [], "end_us": [], "queue": r.get("Queue_Id", r.get("Stream_Id", "?"))})
        d["start_us"].append((int(r["Start_Timestamp"]) - t0) / 1e3)
        d["dur_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        d["end_us"].append((int(r["End_Timestamp"]) - t0) / 1e3)
out = {"trace": os.path.relpath(f), "calls": len(calls), "span_us_mean": float(np.mean(spans)),
       "span_us_pct": [float(x) for x in np.percentile(spans, [5, 50, 95])], "launches": {}}
for k, d in sorted(per.items(), key=lambda kv: np.mean(kv[1]["start_us"])):
    out["launches"][k] = {"queue": d["queue"], "n": len(d["dur_us"]), "start_us": round(float(np.mean(d["start_us"])), 2),
                          "dur_us": round(float(np.mean(d["dur_us"])), 2), "end_us": round(float(np.mean(d["end_us"])), 2)}
print(json.dumps(out, indent=1))
if a.json:
    json.dump(out, open(a.json, "w"), indent=1)
