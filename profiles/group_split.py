"""Cost split of the sorted-group kernel k_stage1g: run stage 1 with only the ORD / ORDV
factors (k_stage1g<G_ORD>), only the LVL / PDF factors (k_stage1g<G_LVL>, with and
without doc_pdf), and all of them (k_stage1g<G_OL>), three times each; run under
`rocprofv3 --kernel-trace --stats` for the per-launch durations.
    python profiles/group_split.py [S] [D]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "replication-of-minute-frequency-factor_amd"))

import torch  # noqa: E402

from mff import catalog, engine, synth  # noqa: E402

SETS = {
    "LVLONLY_NOPDF": ["doc_kurt"],
    "ORD": ["mmt_top50VolumeRet", "mmt_bottom50VolumeRet", "mmt_top20VolumeRet", "mmt_bottom20VolumeRet",
            "doc_vol10_ratio", "doc_vol5_ratio", "doc_vol50_ratio"],
    "LVL": ["doc_kurt", "doc_skew", "doc_std"],
    "LVLPDF": ["doc_kurt", "doc_skew", "doc_std", "doc_pdf60", "doc_pdf70", "doc_pdf80", "doc_pdf90", "doc_pdf95"],
    "ALL": list(catalog.NAMES),
}


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    D = int(sys.argv[2]) if len(sys.argv) > 2 else 500
    dev = torch.device("cuda:0")
    bars, mask = synth.make_panel_device(S, D, dev, config=4)
    panel = engine.DevicePanel(bars, mask)
    only = os.environ.get("SPLIT_SET")
    for tag, names in SETS.items():
        if only and tag != only:
            continue
        ts = []
        for _ in range(4):
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            r = engine.compute_factors(panel, names, events=ev)
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]))
            del r
        print(tag, "pass ms", [round(t, 3) for t in ts[1:]], flush=True)


if __name__ == "__main__":
    main()
