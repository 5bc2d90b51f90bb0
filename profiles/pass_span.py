"""Per-pass span of the stage-1 launches from a rocprofv3 kernel trace.

The stage-1 pass runs its launches on three streams (the high / low serial kernel from
the pass start, the sorted-group and wave-pair kernels on the launch stream, the doc_pdf
sort / count on a side stream), so the per-kernel averages of `--stats` overlap and do
not add up to the pass; the pass time bench.py's HIP events measure is the span from the
first launch's start to the last launch's end.  This groups the trace's stage-1 /
doc_pdf dispatches into passes (one k_stage1g launch per pass; the high / low kernel
goes with the group launch nearest its start) and writes one row per pass: span, and
each kernel's duration.

    python profiles/pass_span.py <trace_dir> <out.csv>
"""
import csv
import glob
import os
import sys


def main():
    src, out = sys.argv[1], sys.argv[2]
    files = glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel trace under {src}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"]
                if "k_stage1" in name or "k_pdf_" in name:
                    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    short = lambda n: n.split("(")[0].replace("void ", "").split("::")[-1]
    g = [st for st, _, n in rows if short(n).startswith("k_stage1g")]
    if not g:
        raise SystemExit("no k_stage1g launch in the trace")
    passes = [{"start": s0, "end": s0, "kernels": {}} for s0 in g]
    for st, en, name in rows:
        k = short(name)
        if k.startswith("k_stage1s<18"):  # launched on its own stream just before the group kernel
            i = min(range(len(g)), key=lambda q: abs(g[q] - st))
        else:
            i = max(q for q in range(len(g)) if g[q] <= st) if st >= g[0] else 0
        p = passes[i]
        p["kernels"][k] = (st, en)
        p["start"] = min(p["start"], st)
        p["end"] = max(p["end"], en)
    names = sorted({k for p in passes for k in p["kernels"]})
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["pass", "span_ms"] + [f"{k}_ms" for k in names])
        for i, p in enumerate(passes):
            w.writerow([i, round((p["end"] - p["start"]) / 1e6, 3)]
                       + [round((p["kernels"][k][1] - p["kernels"][k][0]) / 1e6, 3) if k in p["kernels"] else ""
                          for k in names])
    for i, p in enumerate(passes):
        print(f"pass {i}: span {(p['end'] - p['start']) / 1e6:.3f} ms, {len(p['kernels'])} launches")
        for k, (st, en) in sorted(p["kernels"].items(), key=lambda kv: kv[1][0]):
            print(f"    {k:32s} {(st - p['start']) / 1e6:8.3f} -> {(en - p['start']) / 1e6:8.3f} ms")


if __name__ == "__main__":
    main()
