#!/usr/bin/env python3
"""Basic-block instruction counts of one kernel in a gfx950 assembly listing (hipcc -S --cuda-device-only).

  python tools/asm_blocks.py listing.s KERNEL_SUBSTRING [--min 20]

Prints each block's label, its VALU / SALU / LDS / VMEM / other counts and the branch that ends it
(backward branches mark loops), so a kernel's per-pixel loop can be sized without a profiler."""
import re
import sys


def kernel_lines(path, name):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and name in l.split(":")[0])
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end]


def classify(op):
    if op.startswith(("v_",)):
        return "valu"
    if op.startswith(("s_waitcnt", "s_barrier", "s_nop", "s_sleep", "s_setprio")):
        return "sync"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 0
    lines = kernel_lines(path, name)
    blocks, cur = [], {"label": "entry", "n": {}, "end": "", "idx": 0}
    labels = {}
    for l in lines:
        s = l.strip()
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            blocks.append(cur)
            cur = {"label": m.group(1), "n": {}, "end": "", "idx": len(blocks)}
            labels[m.group(1)] = len(blocks)
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        c = classify(op)
        cur["n"][c] = cur["n"].get(c, 0) + 1
        if c == "branch":
            cur["end"] = s
    blocks.append(cur)
    tot = {}
    for b in blocks:
        for k, v in b["n"].items():
            tot[k] = tot.get(k, 0) + v
        size = sum(b["n"].values())
        if size < mn:
            continue
        back = ""
        m = re.search(r"(\.LBB\S+)", b["end"])
        if m and labels.get(m.group(1), 1 << 30) <= b["idx"]:
            back = f"  <-- loop back to {m.group(1)}"
        print(f"{b['label']:<16} {size:5d}  " + " ".join(f"{k}={v}" for k, v in sorted(b["n"].items())) + back)
    print("total", tot)


if __name__ == "__main__":
    main()
