#!/usr/bin/env python3
"""TEST INFRASTRUCTURE ONLY. Writes a SCRATCH copy of the reference's parallel.cpp whose
two scene initialisers (`s_Spheres`, parallel.cpp:15-26; `s_SphereMats`, :40-51) hold
learnraytracing_amd.scene.random_scene(N, seed) instead of the 9 default spheres, so the
reference's own HitWorld / Scatter / Trace (whose kSphereCount is the compile-time size
of that array, parallel.cpp:27) run the 1000-sphere scene of BASELINE configs 4-5.

    python3 oracle/gen_ref_scene.py OUTDIR [N] [SEED]

Only the two initialiser bodies change; every other byte of the reference file is kept.
The copy goes to OUTDIR (a /tmp path, see oracle/Makefile `ref1000`) and is never
committed: oracle/Makefile compiles ref_harness.cpp with -IOUTDIR ahead of the reference
directory, so `#include "parallel.cpp"` picks the copy and everything else resolves to
/root/reference/src/cpu as for libref.so. Values are written as exact hexadecimal float
literals (the scene's float32 values, bit for bit).
"""
from __future__ import annotations

import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
REF = os.environ.get("REF", "/root/reference/src/cpu")
sys.path.insert(0, ROOT)


def hexf(v: float) -> str:
    return "0.0f" if v == 0 else float(v).hex() + "f"


def f3(v) -> str:
    return f"float3({hexf(v.x)}, {hexf(v.y)}, {hexf(v.z)})"


def main():
    out = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    from learnraytracing_amd.scene import random_scene
    sph, mat = random_scene(n, seed)
    src = open(os.path.join(REF, "parallel.cpp"), "rb").read().decode("latin-1")
    types = ["Material::Lambert", "Material::Metal", "Material::Dielectric"]
    sbody = "\n".join(f"\t{{ {f3(s.center)}, {hexf(s.radius)} }}," for s in sph)
    mbody = "\n".join(f"\t{{ {types[m.type]}, {f3(m.albedo)}, {f3(m.emissive)}, {hexf(m.roughness)}, {hexf(m.ri)} }},"
                      for m in mat)
    pat_s = re.compile(r"(static Sphere s_Spheres\[\]\s*=\s*\{)(.*?)(\n\};)", re.S)
    pat_m = re.compile(r"(static Material s_SphereMats\[kSphereCount\]\s*=\s*\{)(.*?)(\n\};)", re.S)
    if not pat_s.search(src) or not pat_m.search(src):
        raise SystemExit("gen_ref_scene: scene initialisers not found in the reference parallel.cpp")
    src = pat_s.sub(lambda m: m.group(1) + "\n" + sbody + m.group(3), src, count=1)
    src = pat_m.sub(lambda m: m.group(1) + "\n" + mbody + m.group(3), src, count=1)
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "parallel.cpp"), "wb") as f:
        f.write(src.encode("latin-1"))
    print(f"gen_ref_scene: {out}/parallel.cpp with random_scene({n}, {seed})")


if __name__ == "__main__":
    main()
