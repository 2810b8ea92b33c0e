#!/usr/bin/env python3
"""Summarise an LRT_EXP_WAVETRACE dump (tools/build_variant.sh WT -DLRT_EXP_WAVETRACE;
LRT_WAVETRACE=<file> python bench.py ...): wave lifetimes and how many waves were
resident over the launch, for the LAST launch in the file.

    python tools/wavetrace.py <file> [bins]
"""
import sys

import numpy as np


def launches(path):
    raw = np.fromfile(path, dtype=np.uint64)
    i, out = 0, []
    while i < len(raw):
        n = int(raw[i])
        out.append(raw[i + 1:i + 1 + 4 * n].reshape(n, 4))
        i += 1 + 4 * n
    return out


def main():
    ls = launches(sys.argv[1])
    bins = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    w = ls[-1].astype(np.int64)
    t0, t1 = w[:, 0], w[:, 1]
    base = t0.min()
    t0, t1 = (t0 - base) * 10.0, (t1 - base) * 10.0        # 100 MHz ticks -> ns
    span = t1.max()
    dur = t1 - t0
    xcc = (w[:, 2] >> 32) & 0xF
    ntask = w[:, 2] >> 40
    tl = (w[:, 3] - base) * 10.0                          # the last task's start (pool kernel)
    print(f"launches in file {len(ls)}; last: {len(w)} waves, span {span / 1e3:.1f} us")
    print(f"wave lifetime us: mean {dur.mean() / 1e3:.1f}  p10 {np.percentile(dur, 10) / 1e3:.1f}  "
          f"p50 {np.percentile(dur, 50) / 1e3:.1f}  p90 {np.percentile(dur, 90) / 1e3:.1f}  max {dur.max() / 1e3:.1f}")
    print(f"wave-us / (span * 1024 SIMDs) = mean resident waves per SIMD {dur.sum() / span / 1024:.2f}")
    edges = np.linspace(0, span, bins + 1)
    res = []
    for a, b in zip(edges[:-1], edges[1:]):
        ov = np.clip(np.minimum(t1, b) - np.maximum(t0, a), 0, None).sum() / (b - a) / 1024
        res.append(ov)
    print("resident waves/SIMD per time bin:", " ".join(f"{r:.1f}" for r in res))
    if ntask.max() > 0:
        last = t1 - tl
        print(f"tasks per wave: mean {ntask.mean():.2f}  min {ntask.min()}  max {ntask.max()}")
        print(f"last task us: mean {last.mean() / 1e3:.1f}  p10 {np.percentile(last, 10) / 1e3:.1f}  "
              f"p50 {np.percentile(last, 50) / 1e3:.1f}  p90 {np.percentile(last, 90) / 1e3:.1f}; "
              f"last start p10 {np.percentile(tl, 10) / 1e3:.1f} p90 {np.percentile(tl, 90) / 1e3:.1f}")
        print(f"wave end us: p10 {np.percentile(t1, 10) / 1e3:.1f}  p50 {np.percentile(t1, 50) / 1e3:.1f}  "
              f"p90 {np.percentile(t1, 90) / 1e3:.1f}")
    for x in np.unique(xcc):
        m = xcc == x
        print(f"  xcc {x}: waves {m.sum():6d}  last end {t1[m].max() / 1e3:7.1f} us  first start {t0[m].min() / 1e3:6.1f} us")


if __name__ == "__main__":
    main()
