"""Kernel resource table of one translation unit (VGPRs, spills, scratch, occupancy).

    python tools/resusage.py lrt_pool_d8 [-DNAME=VALUE ...] [--filter SUBSTR]

Compiles learnraytracing_amd/csrc/<unit>.hip for the device only with
-Rpass-analysis=kernel-resource-usage (make isa) and prints one line per kernel.
"""
import re
import subprocess
import sys
from pathlib import Path

CSRC = Path(__file__).resolve().parent.parent / "learnraytracing_amd" / "csrc"


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names),
                         capture_output=True, text=True).stdout.split("\n")
    return out[:len(names)]


def main():
    args = sys.argv[1:]
    filt = None
    if "--filter" in args:
        i = args.index("--filter")
        filt = args[i + 1]
        del args[i:i + 2]
    unit, defs = args[0], args[1:]
    r = subprocess.run(["make", "-s", "-B", "isa", f"U={unit}", "EXTRA=" + " ".join(defs)], cwd=CSRC,
                       capture_output=True, text=True)
    text = r.stdout + r.stderr
    if r.returncode:
        sys.exit(text[-3000:])
    rows, cur = [], None
    for line in text.splitlines():
        m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]"
                      r"|SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]): (\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k.split(" [")[0]] = v
    names = demangle([r["name"] for r in rows])
    print(f"{'VGPR':>4} {'vspill':>6} {'sspill':>6} {'scratch':>7} {'occ':>3}  kernel")
    for r, n in zip(rows, names):
        n = n.replace("lrt::", "").replace("(lrt::KernelArgs)", "")
        if filt and filt not in n:
            continue
        print(f"{r.get('VGPRs', '?'):>4} {r.get('VGPRs Spill', '?'):>6} {r.get('SGPRs Spill', '?'):>6} "
              f"{r.get('ScratchSize', '?'):>7} {r.get('Occupancy', '?'):>3}  {n}")


if __name__ == "__main__":
    main()
