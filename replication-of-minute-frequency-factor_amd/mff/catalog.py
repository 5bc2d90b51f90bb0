"""Factor catalogue: the 58 stage-1 outputs in reference order.

Ids are the row index of the device output ``val[F][D][S]`` when all factors are
requested and match ``include/mff.h`` (``MFF_F_*``).  Names are the reference
output column names (``cal_<name>`` in MinuteFrequentFactorCalculateMethodsCICC.py,
cited ``CM:<line>``).  ``FAMILY`` groups factors by the kernel section that computes
them (SURVEY.md §8(a) "Fam" column); ``FIELDS`` says which OHLCV planes a family reads,
so a factor subset only streams the planes it needs (SURVEY §8(d) "32 + 960·|φ| + 9·|F′|").
"""
from __future__ import annotations

from typing import Dict, List, Sequence

# (name, reference line of the def, family)
_TABLE = [
    ("mmt_pm", 12, "SEG"),
    ("mmt_last30", 27, "SEG"),
    ("mmt_paratio", 42, "SEG"),
    ("mmt_am", 63, "SEG"),
    ("mmt_between", 78, "SEG"),
    ("mmt_ols_qrs", 93, "OLS"),
    ("mmt_ols_corr_square_mean", 176, "OLS"),
    ("mmt_ols_corr_mean", 225, "OLS"),
    ("mmt_ols_beta_mean", 274, "OLS"),
    ("mmt_ols_beta_zscore_last", 327, "OLS"),
    ("mmt_top50VolumeRet", 379, "ORD"),
    ("mmt_bottom50VolumeRet", 405, "ORD"),
    ("mmt_top20VolumeRet", 431, "ORD"),
    ("mmt_bottom20VolumeRet", 457, "ORD"),
    ("vol_volume1min", 485, "MOMV"),
    ("vol_range1min", 499, "MOMH"),
    ("vol_return1min", 518, "MOMR"),
    ("vol_upVol", 537, "MOMR"),
    ("vol_upRatio", 563, "MOMR"),
    ("vol_downVol", 591, "MOMR"),
    ("vol_downRatio", 617, "MOMR"),
    ("shape_skew", 647, "MOMR"),
    ("shape_kurt", 660, "MOMR"),
    ("shape_skratio", 673, "MOMR"),
    ("shape_skewVol", 690, "MOMV"),
    ("shape_kurtVol", 703, "MOMV"),
    ("shape_skratioVol", 716, "MOMV"),
    ("liq_amihud_1min", 734, "SUMC"),
    ("liq_closeprevol", 764, "SUMV"),
    ("liq_closevol", 778, "SUMV"),
    ("liq_firstCallR", 792, "SUMV"),
    ("liq_lastCallR", 805, "SUMV"),
    ("liq_openvol", 823, "SUMV"),
    ("corr_prv", 836, "CORR"),
    ("corr_prvr", 850, "CORR"),
    ("corr_pv", 877, "CORR"),
    ("corr_pvd", 891, "CORR"),
    ("corr_pvl", 905, "CORR"),
    ("corr_pvr", 919, "CORR"),
    ("doc_kurt", 937, "LVL"),
    ("doc_skew", 960, "LVL"),
    ("doc_std", 983, "LVL"),
    ("doc_pdf60", 1006, "PDF"),
    ("doc_pdf70", 1033, "PDF"),
    ("doc_pdf80", 1060, "PDF"),
    ("doc_pdf90", 1087, "PDF"),
    ("doc_pdf95", 1114, "PDF"),
    ("doc_vol10_ratio", 1141, "ORDV"),
    ("doc_vol5_ratio", 1162, "ORDV"),
    ("doc_vol50_ratio", 1183, "ORDV"),
    ("trade_bottom20retRatio", 1206, "TRD"),
    ("trade_bottom50retRatio", 1227, "TRD"),
    ("trade_headRatio", 1251, "SUMV"),
    ("trade_tailRatio", 1280, "SUMV"),
    ("trade_top20retRatio", 1309, "TRD"),
    ("trade_top50retRatio", 1331, "TRD"),
    ("trade_topNeg20retRatio", 1353, "TRD"),
    ("trade_topPos20retRatio", 1381, "TRD"),
]

NAMES: List[str] = [t[0] for t in _TABLE]
REF_LINE: Dict[str, int] = {t[0]: t[1] for t in _TABLE}
FAMILY: Dict[str, str] = {t[0]: t[2] for t in _TABLE}
ID: Dict[str, int] = {n: i for i, n in enumerate(NAMES)}
N_FACTORS = len(NAMES)
assert N_FACTORS == 58

# field planes: 0 open, 1 high, 2 low, 3 close, 4 volume
FIELD_NAMES = ["open", "high", "low", "close", "volume"]
FIELDS = {
    "SEG": (0, 3), "OLS": (1, 2), "ORD": (0, 3, 4), "MOMV": (4,), "MOMH": (1, 2),
    "MOMR": (0, 3), "SUMC": (3, 4), "SUMV": (4,), "CORR": (3, 4), "LVL": (3, 4),
    "PDF": (3, 4), "ORDV": (4,), "TRD": (0, 3, 4),
}

PDF_IDS = [ID[f"doc_pdf{p}"] for p in (60, 70, 80, 90, 95)]
# the five calls built on rolling(index_column='minute_in_trade') (CM:114-118): a frame
# whose minute_in_trade decreases inside a stock-day makes exactly these calls raise
OLS_NAMES = [n for n in NAMES if FAMILY[n] == "OLS"]
OLS_IDS = [ID[n] for n in OLS_NAMES]


def resolve(names: Sequence[str] | None) -> List[int]:
    """Factor names (with or without the ``cal_`` prefix) -> catalogue ids."""
    if names is None:
        return list(range(N_FACTORS))
    out = []
    for n in names:
        n = n[4:] if n.startswith("cal_") else n
        if n not in ID:
            raise KeyError(f"unknown factor {n!r}")
        out.append(ID[n])
    return out


def fields_for(ids: Sequence[int]) -> List[int]:
    need = set()
    for i in ids:
        need.update(FIELDS[FAMILY[NAMES[i]]])
    return sorted(need)


def algorithmic_bytes_per_stock_day(ids: Sequence[int]) -> int:
    """32 B mask + 960 B per field plane read + 9 B per output."""
    return 32 + 960 * len(fields_for(ids)) + 9 * len(ids)
