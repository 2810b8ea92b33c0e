#!/usr/bin/env python3
"""Print per-launch averages of every counter in <dir>/<kernel>_g*_counter_collection.csv."""
import csv, collections, glob, os, sys
d = sys.argv[1]
table = collections.defaultdict(dict)
for f in sorted(glob.glob(os.path.join(d, "*_g*_counter_collection.csv"))):
    k = os.path.basename(f).split("_g")[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if any(s in r["Kernel_Name"] for s in ("paths", "trace_kernel", "regen_kernel")):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for c, v in agg.items():
        table[c][k] = sum(v) / len(v)
ks = sorted({k for v in table.values() for k in v})
print("counter".ljust(28) + "".join(k.rjust(14) for k in ks))
for c in sorted(table):
    print(c.ljust(28) + "".join(("%.4g" % table[c].get(k, float("nan"))).rjust(14) for k in ks))
