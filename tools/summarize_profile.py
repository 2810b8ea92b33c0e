#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output for trace_kernel into profiles/<run>/summary.json and
(optionally) record the HBM traffic per launch in profiles/pmc_traffic.json, which
bench.py reads for its roofline.traffic field.

    python tools/summarize_profile.py <prof_dir> <out_dir> [--traffic-key config2_n1]

Traffic correction (MI355X_MICROARCH.md §HBM, gfx950): FETCH_SIZE reports half the
bytes of wide (16 B/lane) coalesced streaming reads, so bytes_read = 2 * FETCH_SIZE KiB;
WRITE_SIZE is exact for 16-B-per-lane stores. Counters were collected in separate
--pmc passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNEL = "trace_kernel"


def per_launch(pattern):
    vals = defaultdict(list)
    meta = {}
    for f in glob.glob(pattern):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta = {k: r[k] for k in ("Kernel_Name", "Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                                          "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count")}
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}, meta


def main():
    prof, out = sys.argv[1], sys.argv[2]
    key = sys.argv[sys.argv.index("--traffic-key") + 1] if "--traffic-key" in sys.argv else None
    os.makedirs(out, exist_ok=True)
    summary = {"kernel": KERNEL}
    # trace_*: the bench's default command (consecutive launches overlap on 2 streams);
    # trace1_*: the same with --streams 1, each launch alone -- its duration prices the
    # VALU issue rate of the PMC passes (counter collection serialises launches too)
    for name, field in (("trace_kernel_stats.csv", "kernel_trace"), ("trace1_kernel_stats.csv", "kernel_trace_serial")):
        f = os.path.join(prof, name)
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Name"]:
                summary[field] = {"name": r["Name"], "calls": int(r["Calls"]),
                                  "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                                  "max_ns": float(r["MaxNs"]), "percent": float(r["Percentage"])}
    counters, n, meta = per_launch(os.path.join(prof, "pmc_*counter_collection.csv"))
    summary["launch"] = meta
    summary["counters_per_launch"] = counters
    summary["launches_sampled"] = n
    if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
        rd = 2.0 * counters["FETCH_SIZE"] * 1024
        wr = counters["WRITE_SIZE"] * 1024
        summary["hbm_bytes_per_launch"] = {"read_corrected": rd, "write": wr, "total": rd + wr,
                                           "raw_fetch_size_kib": counters["FETCH_SIZE"],
                                           "raw_write_size_kib": counters["WRITE_SIZE"]}
        if key:
            p = os.path.join(os.path.dirname(out.rstrip("/")), "pmc_traffic.json")
            d = json.load(open(p)) if os.path.exists(p) else {}
            d[key] = {"bytes_per_launch": rd + wr, "source": os.path.relpath(out, os.path.dirname(p))}
            json.dump(d, open(p, "w"), indent=1)
    if "SQ_INSTS_VALU" in counters and "SQ_WAVES" in counters:
        summary["valu_wave_instructions_per_wave"] = counters["SQ_INSTS_VALU"] / counters["SQ_WAVES"]
        kt = summary.get("kernel_trace_serial") or summary.get("kernel_trace")
        if kt:
            t = kt["avg_ns"] * 1e-9
            # 256 CUs x 4 SIMD, one wave64 VALU instruction per 2 cycles per SIMD at 2.4 GHz
            peak = 256 * 4 * 2.4e9 / 2
            summary["valu_issue_rate"] = counters["SQ_INSTS_VALU"] / t
            summary["valu_issue_frac_of_peak"] = counters["SQ_INSTS_VALU"] / t / peak
    json.dump(summary, open(os.path.join(out, "summary.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
