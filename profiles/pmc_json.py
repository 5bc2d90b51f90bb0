"""profiles/pmc_stage1.json from the rocprofv3 --pmc pass directories of profiles/gpu_pmc.sh
(one bench step, warmup 0: exactly one stage-1 pass per dispatch set).

    python profiles/pmc_json.py DIR STOCKS DAYS ROUND [out.json]

HBM bytes follow MI355X_MICROARCH.md's HBM section: FETCH_SIZE (KiB) x 2 on gfx950 for
wide streaming reads (it tallies 128-B requests at 64 B) + WRITE_SIZE (KiB, exact for
16-B-per-lane stores).  The guide leaves other access shapes to a calibration on a known
byte count: the serial kernels (k_stage1s*, the wave pair) stage rows by LDS-DMA in 64-B
pieces (16 rows x 64 B per wave-instruction), for which FETCH_SIZE reports 0.83 of the
bytes read (profiles/ubench/rowload.hip kernel D: 1.986 GB counted for 2.400 GB read,
profiles/r04c/fetch_calib.log), so their FETCH_SIZE is scaled by 2.400 / 1.986.  Per kernel: the counters summed over its dispatches in the pass,
VALU wave-instructions per stock-day, f64 share, and the wave-cycle split (waiting /
issue-stalled / VALU-active, SQ_* quad-cycles)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

PASS = ("k_stage1", "k_pdf_sort", "k_pdf_count")  # the launches of one stage-1 pass
DMA64 = 2.400 / 1.986  # FETCH_SIZE -> bytes for the 64-B LDS-DMA row pieces (calibrated)


def fetch_factor(name):
    """FETCH_SIZE correction of a kernel: the serial kernels' LDS-DMA pieces (calibrated),
    else the guide's x 2 for wide streaming reads."""
    return DMA64 if name.startswith("k_stage1s") else 2.0
F64 = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")


def main():
    root, S, D, rnd = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                             "pmc_stage1.json")
    tab = defaultdict(lambda: defaultdict(float))
    for path in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"].split("(")[0].replace("void ", "").replace("mff::", "")
                name = name.replace("s1s::", "").replace("g16::", "")
                if not any(p in name for p in PASS):
                    continue
                tab[name][row["Counter_Name"]] += float(row["Counter_Value"])
    sd = S * D
    per, tot = {}, defaultdict(float)
    for k, cs in sorted(tab.items()):
        e = dict(cs)
        hbm = 1024.0 * (fetch_factor(k) * cs.get("FETCH_SIZE", 0.0) + cs.get("WRITE_SIZE", 0.0))
        e["hbm_bytes"] = hbm
        e["fetch_factor"] = round(fetch_factor(k), 4)
        n = cs.get("SQ_INSTS_VALU", 0.0)
        f64 = sum(cs.get(c, 0.0) for c in F64)
        wc = cs.get("SQ_WAVE_CYCLES", 0.0)
        e["valu_per_stock_day"] = round(n / sd, 1)
        e["f64_share"] = round(f64 / n, 3) if n else None
        if wc:
            e["wait_frac"] = round(cs.get("SQ_WAIT_ANY", 0.0) / wc, 3)
            e["issue_stall_frac"] = round(cs.get("SQ_WAIT_INST_ANY", 0.0) / wc, 3)
            e["valu_active_frac"] = round(cs.get("SQ_ACTIVE_INST_VALU", 0.0) / wc, 3)
        per[k] = e
        for c, v in cs.items():
            tot[c] += v
    res = {
        "kernel": "stage-1 pass: every k_stage1* launch of one bench step + the doc_pdf sort / count",
        "stocks": S, "days": D, "round": rnd,
        "fetch_size_kib": tot.get("FETCH_SIZE"), "write_size_kib": tot.get("WRITE_SIZE"),
        "hbm_bytes_per_launch": sum(e["hbm_bytes"] for e in per.values()),
        "hbm_bytes_calibrated": sum(e["hbm_bytes"] for e in per.values()),
        "hbm_bytes_uncalibrated_x2": 1024.0 * (2.0 * tot.get("FETCH_SIZE", 0.0) + tot.get("WRITE_SIZE", 0.0)),
        "fetch_calibration": "profiles/r04c/fetch_calib.log (64-B LDS-DMA pieces: x %.4f)" % DMA64,
        "sq": {k: v for k, v in tot.items() if not k.endswith("_SIZE")},
        "per_kernel": per,
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    n = tot.get("SQ_INSTS_VALU", 0.0)
    print(f"VALU per stock-day {n / sd:.1f}; HBM bytes per pass {res['hbm_bytes_per_launch'] / 1e9:.2f} GB")
    for k, e in per.items():
        print(f"{k:40s} valu/sd {e['valu_per_stock_day']:7.1f} f64 {e['f64_share']} wait {e.get('wait_frac')} "
              f"stall {e.get('issue_stall_frac')} valu-active {e.get('valu_active_frac')} hbm {e['hbm_bytes'] / 1e9:.2f} GB")


if __name__ == "__main__":
    main()
