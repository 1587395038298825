#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes: per-dispatch average of every counter for kernels matching a pattern."""
import csv, glob, json, os, sys, collections
d = sys.argv[1]; pat = sys.argv[2] if len(sys.argv) > 2 else "trace_"
agg = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (disp, name), v in per.items():
        agg[name].append(v)
out = {k: sum(v) / len(v) for k, v in sorted(agg.items())}
print(json.dumps(out, indent=1))
