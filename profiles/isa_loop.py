"""Static instruction histogram of the innermost loop that holds a marker instruction.

usage: python profiles/isa_loop.py file.s kernel_symbol [marker=ds_read_b128]
Counts instructions in the basic blocks that LLVM annotates as members of the loop
(";   in Loop: Header=BBx_y" / ";   Parent Loop ..." headers) containing the first
occurrence of the marker in the kernel.  Used to compare per-chunk VALU counts of
the serial kernels between builds.
"""
import re
import sys
from collections import Counter


def main():
    path, sym = sys.argv[1], sys.argv[2]
    marker = sys.argv[3] if len(sys.argv) > 3 else "ds_read_b128"
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    blocks, cur, hdr = [], None, None
    for l in lines[start:end]:
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):\s*(;.*)?$", l)
        if m:
            label = m.group(1)
            comment = m.group(2) or ""
            h = re.search(r"Header=(BB\d+_\d+)", comment)
            hdr = h.group(1) if h else None
            cur = [label, hdr, []]
            blocks.append(cur)
            continue
        if cur is not None:
            if "Loop Header" in l and not cur[2]:
                cur[1] = cur[0].lstrip(".L")
            cur[2].append(l)
    # loop of the marker
    loop = None
    for label, hdr, body in blocks:
        if any(marker in x for x in body):
            loop = hdr
            break
    if loop is None:
        print("marker not in a loop")
        return
    c = Counter()
    for label, hdr, body in blocks:
        if hdr == loop or label.lstrip(".L") == loop:
            for x in body:
                t = x.strip().split()
                if t and re.match(r"^[vsdgb][a-z0-9_]*$", t[0]) and not t[0].startswith(";"):
                    op = re.sub(r"_e(32|64)$", "", t[0])
                    c[op] += 1
    valu = sum(v for k, v in c.items() if k.startswith("v_"))
    salu = sum(v for k, v in c.items() if k.startswith("s_"))
    print(f"loop {loop}: VALU {valu}  SALU {salu}  marker count {c.get(marker, 0)}")
    for k, v in c.most_common(24):
        print(f"  {v:5d} {k}")


if __name__ == "__main__":
    main()
