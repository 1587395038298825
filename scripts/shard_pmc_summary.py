#!/usr/bin/env python3
"""Per-round sums of the PMC counters of scripts/shard_pmc_run.py's last
ROUNDS x N tracer dispatches (rocprofv3 --pmc passes p1..pK of one run
directory), the kernel time from the pass's kernel trace, and the derived
fractions of scripts/collect_profiles.py (HBM bytes = 2 x FETCH_SIZE +
WRITE_SIZE KiB, MI355X_MICROARCH.md; VALU issue = SQ_INSTS_VALU x 2 cycles
over 1024 SIMDs x kernel cycles at 2.4 GHz; wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES).
Usage: shard_pmc_summary.py DIR N ROUNDS  -> one JSON object"""
import collections
import csv
import glob
import json
import os
import sys

d, n, rounds = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
tot = collections.defaultdict(float)
kernel_us = []
for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "trace_" in r["Kernel_Name"]:
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    last = sorted(per)[-n * rounds:]
    for disp in last:
        for k, v in per[disp].items():
            tot[k] += v / rounds
    kt = glob.glob(os.path.join(os.path.dirname(f), "*kernel_trace.csv"))
    if kt:
        rows = [r for r in csv.DictReader(open(kt[0])) if "trace_" in r["Kernel_Name"]]
        rows = rows[-n * rounds:]
        kernel_us.append(sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3 for r in rows) / rounds)
out = dict(sorted(tot.items()))
if kernel_us:
    k_us = sorted(kernel_us)[len(kernel_us) // 2]
    out["kernel_us_sum_per_round"] = k_us
    cycles = k_us * 1e-6 * 2.4e9
    if "SQ_INSTS_VALU" in out:
        out["valu_issue_frac"] = out["SQ_INSTS_VALU"] * 2 / (1024 * cycles)
if "SQ_WAIT_ANY" in out and "SQ_WAVE_CYCLES" in out:
    out["wait_frac"] = out["SQ_WAIT_ANY"] / out["SQ_WAVE_CYCLES"]
if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
    out["hbm_bytes_per_round"] = (2 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024
print(json.dumps(out))
