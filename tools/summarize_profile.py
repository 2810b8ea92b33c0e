#!/usr/bin/env python3
"""Summarise the rocprofv3 output of `tools/gpu.sh trace=C pmc=C,fetch pmc=C,write pmc=C,sq`
for the render kernel (trace_kernel or pool_kernel, whichever the run launched) into
profiles/<run>/summary_c<C>.json and register it in profiles/pmc_index.json, which
bench.py reads for its roofline objects.

    python tools/summarize_profile.py gpurun_out/<tag> profiles/<tag> --config C [--key config2_n1]

Per launch of the render kernel (averaged over the launches of each pass):
  * counters_per_launch: every collected counter;
  * lane_util = SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64): active lanes per VALU
    instruction (both counters in the same quad-cycle unit);
  * lane_ops_per_launch = SQ_INSTS_VALU x 64 x lane_util;
  * hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes). MI355X_MICROARCH.md
    (HBM/rocprofv3): on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads;
    WRITE_SIZE is exact for 16-B-per-lane stores. FETCH_SIZE and WRITE_SIZE were collected
    in separate --pmc passes (they do not fit one TCC pass);
  * kernel_trace: rocprofv3 --kernel-trace --stats of the bench command (one render
    stream); alone_leg: the durations of its launch-alone leg from the kernel trace, which
    must agree with the bench line's ms_per_launch_alone (HIP events) of the same run;
    the counters are priced with that duration.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = ("trace_kernel", "pool_kernel")
KERNEL = None   # the one the profiled run launched (main)


def is_render(name):
    return KERNEL in name if KERNEL else any(k in name for k in KERNELS)


def per_launch(files):
    vals = defaultdict(list)
    meta = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if is_render(r["Kernel_Name"]):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                meta = {k: r[k] for k in ("Kernel_Name", "Grid_Size", "Workgroup_Size", "LDS_Block_Size",
                                          "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count") if k in r}
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}, meta


def main():
    global KERNEL
    prof, out = sys.argv[1], sys.argv[2]
    c = int(sys.argv[sys.argv.index("--config") + 1])
    key = sys.argv[sys.argv.index("--key") + 1] if "--key" in sys.argv else f"config{c}_n1"
    os.makedirs(out, exist_ok=True)
    summary = {"kernel": KERNEL, "config": c, "key": key,
               "recipe": f"tools/gpu.sh trace={c} pmc={c},fetch pmc={c},write pmc={c},sq"}
    # the render kernel the traced bench line names (its DrawTest leg runs trace_kernel too,
    # and at config 2 that leg takes longer than the measured launches)
    for f in glob.glob(os.path.join(prof, f"trace_c{c}_*.log")):
        for line in open(f):
            if line.startswith("{"):
                try:
                    KERNEL = json.loads(line)["config"]["kernel"]
                except (ValueError, KeyError):
                    pass
    for f in glob.glob(os.path.join(prof, "**", f"trace_c{c}_kernel_stats.csv"), recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if is_render(r["Name"])]
        if rows and not KERNEL:   # else the render kernel with the most time
            KERNEL = max(rows, key=lambda r: float(r["Percentage"]))["Name"].split("<")[0].split("::")[-1]
        summary["kernel"] = KERNEL
        for r in rows:
            if KERNEL in r["Name"]:
                summary["kernel_trace"] = {"name": r["Name"], "calls": int(r["Calls"]),
                                           "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                                           "max_ns": float(r["MaxNs"]), "percent": float(r["Percentage"])}
    # the launch-alone leg of the traced bench run, in dispatch order (bench.py, round 6): the W
    # warmup launches, the end-to-end leg's untimed frames in flight and its timed steps, then the
    # alone leg's `steps` launches -- the leg whose HIP-event average the bench line divides by
    bench_line = None
    for f in glob.glob(os.path.join(prof, f"trace_c{c}_*.log")):
        for line in open(f, errors="replace"):
            if line.startswith('{"metric"'):
                bench_line = json.loads(line)
    for f in glob.glob(os.path.join(prof, "**", f"trace_c{c}_kernel_trace.csv"), recursive=True):
        rows = sorted((r for r in csv.DictReader(open(f)) if is_render(r["Kernel_Name"])),
                      key=lambda r: int(r["Start_Timestamp"]))
        if bench_line and bench_line.get("ms_per_launch_alone"):
            e2e = bench_line.get("end_to_end") or {}
            a = bench_line["warmup"] + e2e.get("untimed_steps", 0) + e2e.get("steps", 0)
            d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in rows[a:a + bench_line["steps"]]]
            if d:
                summary["alone_leg"] = {"launches": len(d), "avg_ns": sum(d) / len(d), "min_ns": min(d),
                                        "max_ns": max(d),
                                        "bench_ms_per_launch_alone": bench_line["ms_per_launch_alone"],
                                        "bench_ms_per_step": bench_line["ms_per_step"]}
    files = glob.glob(os.path.join(prof, "**", f"pmc_c{c}_*counter_collection.csv"), recursive=True)
    counters, n, meta = per_launch(files)
    summary["launch"] = meta
    summary["counters_per_launch"] = counters
    summary["launches_sampled"] = n
    if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
        rd = 2.0 * counters["FETCH_SIZE"] * 1024
        wr = counters["WRITE_SIZE"] * 1024
        summary["hbm_bytes_per_launch"] = rd + wr
        summary["hbm_detail"] = {"read_corrected": rd, "write": wr, "raw_fetch_size_kib": counters["FETCH_SIZE"],
                                 "raw_write_size_kib": counters["WRITE_SIZE"]}
    if all(k in counters for k in ("SQ_INSTS_VALU", "SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU")):
        lu = counters["SQ_THREAD_CYCLES_VALU"] / (counters["SQ_ACTIVE_INST_VALU"] * 64)
        summary["lane_util"] = round(lu, 4)
        summary["valu_insts_per_launch"] = counters["SQ_INSTS_VALU"]
        summary["lane_ops_per_launch"] = counters["SQ_INSTS_VALU"] * 64 * lu
        kt = summary.get("alone_leg") or summary.get("kernel_trace")
        if kt:
            t = kt["avg_ns"] * 1e-9
            summary["valu_issue_frac"] = counters["SQ_INSTS_VALU"] / t / (256 * 4 * 2.4e9 / 2)
            summary["valu_lane_frac"] = summary["lane_ops_per_launch"] / t / (256 * 4 * 32 * 2.4e9)
    with open(os.path.join(out, f"summary_c{c}.json"), "w") as f:
        json.dump(summary, f, indent=1)
    idx_path = os.path.join(os.path.dirname(out.rstrip("/")), "pmc_index.json")
    idx = json.load(open(idx_path)) if os.path.exists(idx_path) else {}
    idx[key] = os.path.relpath(os.path.join(out, f"summary_c{c}.json"), os.path.dirname(idx_path))
    with open(idx_path, "w") as f:
        json.dump(idx, f, indent=1, sort_keys=True)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
