"""Turn a profiles/run_profiles.sh output directory into the committed summaries:
profiles/pmc_stage1.json (HBM bytes per stage-1 pass = the sum over its launches incl. the
doc_pdf sort / count, read by
bench.py's roofline "traffic"; per-kernel values alongside) and profiles/<round>/rocprof/
*.csv copies.

HBM bytes = FETCH_SIZE x 2 (gfx950: FETCH_SIZE counts half the bytes of a wide
coalesced stream, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both in KiB per dispatch.
That factor is exact for the 16-lane kernels' 1 KiB coalesced pieces; the lane-per-
stock-day kernels stage 64-B row pieces by LDS-DMA, for which profiles/ubench/rowload.hip
(kD, every byte read once) measures FETCH_SIZE = 0.822 x the bytes read, so
`hbm_bytes_calibrated` uses x 1/0.822 for the k_stage1s launches instead.
    python profiles/summarize.py gpurun_out/prof_r01 r01 --stocks 5000 --days 2500
"""
import argparse
import csv
import json
import os
import shutil

HERE = os.path.dirname(os.path.abspath(__file__))


def counters(path, per_kernel):
    """Sum each counter over the stage-1 launches of the profiled step (one dispatch per
    kernel); per_kernel[name][counter] keeps the split."""
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1]
            if name.startswith("k_stage1") or name.startswith("k_pdf"):
                v = float(row["Counter_Value"])
                out[row["Counter_Name"]] = out.get(row["Counter_Name"], 0.0) + v
                k = per_kernel.setdefault(name, {})
                k[row["Counter_Name"]] = k.get(row["Counter_Name"], 0.0) + v
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("tag")
    ap.add_argument("--stocks", type=int, default=5000)
    ap.add_argument("--days", type=int, default=2500)
    a = ap.parse_args()
    c, per = {}, {}
    for d in sorted(os.listdir(a.src)):
        p = os.path.join(a.src, d, "pmc_counter_collection.csv")
        if d.startswith("pmc_") and os.path.exists(p):
            c.update(counters(p, per))
    fetch_kb, write_kb = c.get("FETCH_SIZE"), c.get("WRITE_SIZE")
    res = {"kernel": "stage-1 pass (all k_stage1* launches of one step + the doc_pdf sort / count "
                     "on the side stream, the launches bench.py's roofline window covers)",
           "stocks": a.stocks, "days": a.days, "round": a.tag,
           "fetch_size_kib": fetch_kb, "write_size_kib": write_kb,
           "hbm_bytes_per_launch": None if fetch_kb is None or write_kb is None
           else int((2 * fetch_kb + write_kb) * 1024),
           "sq": {k: v for k, v in c.items() if k.startswith("SQ_") or k.startswith("GRBM")},
           "per_kernel": {k: {"hbm_bytes": int((2 * v.get("FETCH_SIZE", 0) + v.get("WRITE_SIZE", 0)) * 1024),
                              **v} for k, v in per.items()}}
    cal = 0.0
    for k, v in per.items():
        f = 1.0 / 0.822 if k.startswith("k_stage1s") else 2.0  # k_stage1s incl. k_stage1s_pair
        cal += (f * v.get("FETCH_SIZE", 0.0) + v.get("WRITE_SIZE", 0.0)) * 1024
    res["hbm_bytes_calibrated"] = int(cal)
    with open(os.path.join(HERE, "pmc_stage1.json"), "w") as f:
        json.dump(res, f, indent=1)
    dst = os.path.join(HERE, a.tag.split("-")[0], "rocprof")
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(a.src, "trace", "trace_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
