"""Where a kernel's scratch spills sit: per basic block of the device ISA (make isa U=unit), the
scratch stores/loads, the block's instruction count and its loop depth (LLVM's loop comments).

    python tools/isa_spills.py learnraytracing_amd/csrc/lrt_pool_d8.s 'pool_kernelILi8ELb1ELi2ELi64ELi0E'
"""
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, ln in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(key) + r"\S*:", ln))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur = [], None
    for ln in lines[start:end]:
        m = re.match(r"^(\.LBB\S+|\S+):", ln)
        if m:
            d = re.search(r"Depth=(\d+)", ln)
            cur = {"name": m.group(1), "depth": int(d.group(1)) if d else 0, "st": 0, "ld": 0, "n": 0}
            blocks.append(cur)
            continue
        if cur is None:
            continue
        t = ln.strip()
        if "Loop Depth" in t or "Inner Loop Header" in t:
            d = re.search(r"Depth=(\d+)", t)
            if d:
                cur["depth"] = max(cur["depth"], int(d.group(1)))
        if not t or t[0] in ";.":
            continue
        cur["n"] += 1
        if t.startswith("scratch_store") or t.startswith("buffer_store_dword") and "offen" not in t and "s[0:3]" in t:
            cur["st"] += 1
        if t.startswith("scratch_load"):
            cur["ld"] += 1
    tot = sum(b["n"] for b in blocks)
    print(f"{len(blocks)} blocks, {tot} instructions, scratch stores {sum(b['st'] for b in blocks)} "
          f"loads {sum(b['ld'] for b in blocks)}")
    for b in blocks:
        if b["st"] or b["ld"]:
            print(f"  {b['name']:<14} depth {b['depth']} insts {b['n']:>5} st {b['st']:>3} ld {b['ld']:>3}")


if __name__ == "__main__":
    main()
