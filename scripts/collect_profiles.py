#!/usr/bin/env python3
"""Copy a round's rocprofv3 results from gpurun_out/ into profiles/ (tracked):
kernel-trace stats CSVs, per-dispatch PMC averages, profiles/traffic.json —
HBM bytes per launch keyed by bench workload, computed as the guide prescribes
(MI355X_MICROARCH.md "HBM": FETCH_SIZE/WRITE_SIZE are KiB; gfx950 FETCH_SIZE
counts half of a wide streamed read, so it is doubled) — and profiles/issue.json:
the issue side of the same launches, beside the roofline's brute-force FLOP
fraction (which credits every cull as achieved work):
  valu_issue_frac = SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x kernel cycles at 2.4 GHz)
  wait_frac       = SQ_WAIT_ANY / SQ_WAVE_CYCLES

Usage: python scripts/collect_profiles.py r02 [OUT_DIR]
(OUT_DIR default profiles/; on a GPU box, a directory under gpurun_out/ that
then comes back instead of the raw traces, which exceed gpurun's 64 MiB)
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCENES = {"three_sphere": "three_sphere_scene@1920x1080,depth=5,f32",
          "reflect_refract": "reflect_refract@1920x1080,depth=6,f32",
          "cover": "cover@3840x2160,depth=6,f32",
          "table": "table@3840x2160,depth=6,f32"}


def pmc_means(d, pat="trace_"):
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, name), v in per.items():
            agg[name].append(v)
    return {k: sum(v) / len(v) for k, v in sorted(agg.items())}


def kernel_medians(d):
    """Per-kernel median, mean and count of the dispatch durations (us) in a
    kernel trace: ramp outliers (first launches at low clocks) pull the
    stats CSV's mean above the steady per-launch time."""
    durs = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            durs[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    out = {}
    for k, v in durs.items():
        v.sort()
        out[k] = {"calls": len(v), "median_us": v[len(v) // 2], "mean_us": sum(v) / len(v), "max_us": v[-1]}
    return out


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
    out = os.path.abspath(sys.argv[2]) if len(sys.argv) > 2 else os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)

    def prior(name):  # the tracked file's entries, updated by this round's
        for p in (os.path.join(out, name), os.path.join(ROOT, "profiles", name)):
            if os.path.exists(p):
                return json.load(open(p))
        return {}
    tp, ip = os.path.join(out, "traffic.json"), os.path.join(out, "issue.json")
    traffic, issue = prior("traffic.json"), prior("issue.json")
    for key, workload in SCENES.items():
        src = os.path.join(ROOT, "gpurun_out", f"{rnd}_stats_{key}")
        for f in glob.glob(os.path.join(src, "**", "*kernel_stats.csv"), recursive=True):
            shutil.copy(f, os.path.join(out, f"{rnd}_kernel_stats_{key}.csv"))
        med = kernel_medians(src)
        if med:
            json.dump(med, open(os.path.join(out, f"{rnd}_kernel_medians_{key}.json"), "w"), indent=1)
        log = os.path.join(src, "bench.log")
        if os.path.exists(log):
            lines = [l for l in open(log) if l.startswith("{")]
            if lines:
                open(os.path.join(out, f"{rnd}_bench_under_rocprof_{key}.json"), "w").write(lines[-1])
        m = pmc_means(os.path.join(ROOT, "gpurun_out", f"{rnd}_pmc_{key}"))
        if not m:
            continue
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            hbm = (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024
            m["hbm_bytes_per_launch"] = hbm
            traffic[workload] = hbm
        tracer = [v for k, v in med.items() if "trace_" in k]
        if tracer and "SQ_INSTS_VALU" in m and "SQ_WAVE_CYCLES" in m and "SQ_WAIT_ANY" in m:
            k_us = max(tracer, key=lambda v: v["calls"])["median_us"]  # the bench's kernel
            cycles = k_us * 1e-6 * 2.4e9
            m["valu_issue_frac"] = m["SQ_INSTS_VALU"] * 2 / (1024 * cycles)
            m["wait_frac"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
            issue[workload] = {"valu_issue_frac": m["valu_issue_frac"], "wait_frac": m["wait_frac"],
                               "kernel_us": k_us, "source": f"profiles/{rnd}_pmc_{key}.json"}
        json.dump(m, open(os.path.join(out, f"{rnd}_pmc_{key}.json"), "w"), indent=1)
        print(key, json.dumps(m))
    json.dump(traffic, open(tp, "w"), indent=1)
    json.dump(issue, open(ip, "w"), indent=1)


if __name__ == "__main__":
    main()
