"""Per-section census of a kernel's ISA: VALU instructions by source section and loop.

usage: python profiles/isa_census.py kernel.s kernel_symbol sections.json

The assembly must be built with -g (hipcc -O3 -g -S --cuda-device-only ...): every
instruction is attributed to the `.loc` line in effect; code inlined from a header
(mff_group.h sorts, mff_stats.h moments, ...) is attributed to the section of the last
line of the kernel's own file seen before it (its call site, in program order).
sections.json: {"file": "csrc/mff_stage1g.hip", "sections": [[name, first, last], ...]}
where first / last are line numbers or substrings of the source line that opens / closes
the section (resolved against the source file, so edits do not shift the ranges; with
"ordered": true each opening marker is searched after the previous section's); lines
outside every range count as "other".

Output: per section, VALU in the blocks of each loop (LLVM's "Loop Header" annotations:
the outer per-iteration loop and the nested per-level loops), plus the blocks that only
run on rare paths when marked by a rare-path source line ("rare" ranges in the json), so
a dynamic count = sum(static count x trip count) can be set against the PMC figure.
"""
import json
import re
import sys
from collections import defaultdict


def parse(path, sym):
    lines = open(path).read().split("\n")
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', l)
        if m:
            files[int(m.group(1))] = m.group(3)
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    # to the function's end label (a kernel may hold several s_endpgm)
    end = next((i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end")),
               next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i]))
    blocks = []
    cur = {"label": "entry", "header": None, "depth": 0, "ins": []}
    blocks.append(cur)
    loc = (None, None)
    for l in lines[start:end + 1]:
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):\s*(;.*)?$", l)
        if m:
            comment = m.group(2) or ""
            h = re.search(r"Header=(BB\d+_\d+) Depth=(\d+)", comment)
            d = re.search(r"Loop Header: Depth=(\d+)", comment)
            label = m.group(1).lstrip(".L")
            if d:
                hdr, depth = label, int(d.group(1))
            elif h:
                hdr, depth = h.group(1), int(h.group(2))
            else:
                hdr, depth = None, 0
            cur = {"label": label, "header": hdr, "depth": depth, "ins": []}
            blocks.append(cur)
            continue
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            loc = (files.get(int(m.group(1)), m.group(1)), int(m.group(2)))
            continue
        t = l.strip().split()
        if t and re.match(r"^[vsgb][a-z0-9_]*$", t[0]):
            cur["ins"].append((re.sub(r"_e(32|64)$", "", t[0]), loc))
    return blocks


def main():
    path, sym, spec = sys.argv[1], sys.argv[2], sys.argv[3]
    cfg = json.load(open(spec))
    own = cfg["file"].split("/")[-1]
    import os
    src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "replication-of-minute-frequency-factor_amd", cfg["file"])
    text = open(src).read().split("\n") if os.path.exists(src) else []

    def resolve(x, after=0):
        if isinstance(x, int):
            return x
        for i in range(after, len(text)):
            if x in text[i]:
                return i + 1
        raise SystemExit(f"marker not found: {x!r}")
    secs = []
    prev = 0  # "ordered": each section's opening marker is searched after the previous one
    for name, a, b in cfg["sections"]:
        la = resolve(a, prev if cfg.get("ordered") else 0)
        prev = la
        secs.append([name, la, resolve(b, la) if not isinstance(b, int) else b])
    cfg["sections"] = secs

    def section(line):
        for name, a, b in cfg["sections"]:
            if a <= line <= b:
                return name
        return "other"

    blocks = parse(path, sym)
    table = defaultdict(lambda: defaultdict(int))  # section -> loop header -> VALU
    ctx = "other"
    total = defaultdict(int)
    for b in blocks:
        for op, (f, line) in b["ins"]:
            if f and str(f).split("/")[-1] == own and line:
                ctx = section(line)
            if op.startswith("v_"):
                key = f"{b['header'] or 'straight'} (depth {b['depth']})"
                table[ctx][key] += 1
                total[key] += 1
    print(f"{sym}: static VALU by section and loop")
    for name in [s[0] for s in cfg["sections"]] + ["other"]:
        if name in table:
            parts = ", ".join(f"{k}: {v}" for k, v in sorted(table[name].items()))
            print(f"  {name:28s} {sum(table[name].values()):6d}   {parts}")
    print("  total by loop: " + ", ".join(f"{k}: {v}" for k, v in sorted(total.items())))
    # dynamic estimate: depth-1 blocks once per iteration of the outer loop, depth-2 blocks
    # `inner_trips` times, the prologue (depth 0) once per `outer_trips` iterations;
    # per unit = per iteration / `units_per_iteration`
    dyn = cfg.get("dynamic")
    if dyn:
        per_it = {}
        for name in [s[0] for s in cfg["sections"]] + ["other"]:
            x = 0.0
            for k, v in table.get(name, {}).items():
                depth = int(k.split("depth ")[1].rstrip(")"))
                x += v * (1.0 / dyn["outer_trips"] if depth == 0 else 1.0 if depth == 1 else dyn["inner_trips"])
            per_it[name] = x
        u = dyn["units_per_iteration"]
        tot = sum(per_it.values())
        print(f"dynamic estimate per {dyn['unit']} (depth-2 loops x {dyn['inner_trips']}, prologue / "
              f"{dyn['outer_trips']}; common path, rare branches counted too):")
        for name, x in per_it.items():
            if x:
                print(f"  {name:28s} {x / u:8.1f}   {100.0 * x / tot:5.1f} %")
        print(f"  {'total':28s} {tot / u:8.1f}" + (f"   (PMC: {dyn['pmc']})" if "pmc" in dyn else ""))


if __name__ == "__main__":
    main()
