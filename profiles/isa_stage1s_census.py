"""Per-section VALU census of the one-lane-per-stock-day kernels' bar walks (set H alone,
the wave pair's two waves), per bar of the full-wave walk (the c4 case: every lane has
all 240 bars), from the ISA (profiles/isa_census.py sections, profiles/census_stage1s.json).

usage: python profiles/isa_stage1s_census.py mff_stage1s.s
(hipcc -O3 -g -std=c++17 -S --cuda-device-only --offload-arch=gfx950 csrc/mff_stage1s.hip)

A kernel's bar-walk loops are its loop blocks (LLVM loop annotations) whose bodies hold
the walk's 16-bar chunk; the full-wave walk is the one without the per-quad presence test
(`__builtin_amdgcn_ballot_w64((pm & 0xFu) != 0xFu ...)`, the general walk's) -- i.e. the
loop with the fewest VALU of the kernel's two walks per wave role.  Counts are static
instructions per loop body / 16 bars; branches inside the body (the m <= 50 TRD windows,
the once-per-day snapshots, set H's window tests before bar 49) are counted as if taken,
so the per-bar figure is an upper bound of the dynamic count over the day."""
import collections
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import isa_census as ic  # noqa: E402

KERNELS = {"set H": "_ZN3mff3s1s9k_stage1sILj18ELb1EEEvNS0_5SArgsE",
           "wave pair": "_ZN3mff3s1s14k_stage1s_pairENS0_5SArgsE"}


def main():
    path = sys.argv[1]
    cfg = json.load(open(os.path.join(HERE, "census_stage1s.json")))
    src = open(os.path.join(HERE, "..", "replication-of-minute-frequency-factor_amd", cfg["file"])).read().split("\n")

    def resolve(x, after=0):
        for i in range(after, len(src)):
            if x in src[i]:
                return i + 1
        raise SystemExit(f"marker not found: {x!r}")
    secs, prev = [], 0
    for name, a, b in cfg["sections"]:
        la = resolve(a, prev)
        prev = la
        secs.append((name, la, resolve(b, la)))

    def section(line):
        for name, a, b in secs:
            if a <= line < b:
                return name
        return "other (fmath, headers, loop control)"
    for kname, sym in KERNELS.items():
        blocks = ic.parse(path, sym)
        loops = collections.defaultdict(lambda: collections.defaultdict(collections.Counter))
        quadtest = collections.Counter()
        ctx = "other (fmath, headers, loop control)"
        for b in blocks:
            if not b["header"]:
                continue
            for op, (f, line) in b["ins"]:
                if f and str(f).endswith("mff_stage1s.hip") and line:
                    ctx = section(line)
                    if "ballot_w64((pm & 0xFu) != 0xFu" in src[line - 1]:
                        quadtest[b["header"]] += 1
                if op.startswith("v_"):
                    loops[b["header"]][ctx]["all"] += 1
                    if "f64" in op:
                        loops[b["header"]][ctx]["f64"] += 1
        print(f"== {kname} ({sym})")
        for hdr, tab in sorted(loops.items(), key=lambda x: -sum(v["all"] for v in x[1].values())):
            tot = sum(v["all"] for v in tab.values())
            if tot < 400:
                continue
            kind = "general walk" if quadtest[hdr] else "full-wave walk"
            f64 = sum(v["f64"] for v in tab.values())
            print(f"  loop {hdr} ({kind}): {tot / 16:.1f} VALU per bar ({f64 / 16:.1f} f64)")
            for name, v in sorted(tab.items(), key=lambda x: -x[1]["all"]):
                print(f"    {name:38s} {v['all'] / 16:6.1f}  (f64 {v['f64'] / 16:5.1f})")


if __name__ == "__main__":
    main()
