"""Turn a profiles/run_profiles.sh output directory into the committed summaries:
profiles/pmc_stage1.json (HBM bytes per k_stage1 launch, read by bench.py's roofline
"traffic") and profiles/<round>/rocprof/*.csv copies.

HBM bytes = FETCH_SIZE x 2 (gfx950: FETCH_SIZE counts half the bytes of a wide
coalesced stream, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both in KiB per dispatch.
    python profiles/summarize.py gpurun_out/prof_r01 r01 --stocks 5000 --days 2500
"""
import argparse
import csv
import json
import os
import shutil

HERE = os.path.dirname(os.path.abspath(__file__))


def counters(path):
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Kernel_Name"].startswith("k_stage1"):
                out[row["Counter_Name"]] = float(row["Counter_Value"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("tag")
    ap.add_argument("--stocks", type=int, default=5000)
    ap.add_argument("--days", type=int, default=2500)
    a = ap.parse_args()
    c = {}
    for d in os.listdir(a.src):
        p = os.path.join(a.src, d, "pmc_counter_collection.csv")
        if d.startswith("pmc_") and os.path.exists(p):
            c.update(counters(p))
    fetch_kb, write_kb = c.get("FETCH_SIZE"), c.get("WRITE_SIZE")
    res = {"kernel": "k_stage1", "stocks": a.stocks, "days": a.days, "round": a.tag,
           "fetch_size_kib": fetch_kb, "write_size_kib": write_kb,
           "hbm_bytes_per_launch": None if fetch_kb is None or write_kb is None
           else int((2 * fetch_kb + write_kb) * 1024),
           "sq": {k: v for k, v in c.items() if k.startswith("SQ_") or k.startswith("GRBM")}}
    with open(os.path.join(HERE, "pmc_stage1.json"), "w") as f:
        json.dump(res, f, indent=1)
    dst = os.path.join(HERE, a.tag, "rocprof")
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(a.src, "trace", "trace_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
