"""Parity assertion shared by the GPU tests (tolerance rule C5).

* states (ABSENT / NULL / VALUE) bit-exact;
* among VALUE entries: NaN-ness exact, +-inf exact (sign included);
* finite values: |a - b| <= RTOL * max(|a|, |b|) + ATOL[name].

RTOL = 1e-6 is the north-star tolerance for f64 accumulation over fp32 bars.  ATOL is an
absolute floor for outputs that are differences of nearly equal quantities (skewness of
near-symmetric sets, correlations and sums near zero, products minus one), where both
implementations legitimately differ by f64 rounding of the terms (~1e-16 x term size).
"""
import numpy as np

RTOL = 1e-6
ATOL_DEFAULT = 1e-12
ATOL = {
    # sums / differences of O(1e-3) terms whose result can be ~0
    "mmt_paratio": 1e-12, "trade_bottom20retRatio": 1e-12, "trade_bottom50retRatio": 1e-12,
    "mmt_top50VolumeRet": 1e-12, "mmt_bottom50VolumeRet": 1e-12, "mmt_top20VolumeRet": 1e-12,
    "mmt_bottom20VolumeRet": 1e-12,
    # O(1) statistics that can be ~0
    "shape_skew": 1e-9, "shape_skewVol": 1e-9, "shape_skratio": 1e-9, "shape_skratioVol": 1e-9,
    "doc_skew": 1e-9, "doc_std": 1e-9, "corr_prv": 1e-9, "corr_prvr": 1e-9, "corr_pv": 1e-9,
    "corr_pvd": 1e-9, "corr_pvl": 1e-9, "corr_pvr": 1e-9, "mmt_ols_beta_zscore_last": 1e-9,
    "mmt_ols_corr_mean": 1e-9,
    # ratios of returns to tiny volume shares: terms up to ~1e2
    "trade_top20retRatio": 1e-9, "trade_top50retRatio": 1e-9,
    # qrs: mean of cov**0.5/(var_x var_y) (terms ~1e5) times a z-score
    "mmt_ols_qrs": 1e-6,
}


def compare(gv, gs, ov, os_, name, rtol=RTOL, atol=None):
    """Return a list of human-readable mismatch descriptions (empty = parity)."""
    atol = ATOL.get(name, ATOL_DEFAULT) if atol is None else atol
    gv, gs, ov, os_ = map(np.asarray, (gv, gs, ov, os_))
    bad = []
    st = gs != os_
    if st.any():
        idx = np.argwhere(st)[:5]
        bad.append(f"{name}: {int(st.sum())} state mismatches, e.g. "
                   + ", ".join(f"{tuple(i)} gpu={gs[tuple(i)]} ref={os_[tuple(i)]}" for i in idx))
    m = (os_ == 2) & (gs == 2)
    a, b = gv[m], ov[m]
    an, bn = np.isnan(a), np.isnan(b)
    if (an != bn).any():
        k = np.flatnonzero(an != bn)[:5]
        bad.append(f"{name}: NaN mismatch at {int((an != bn).sum())}: gpu={a[k]} ref={b[k]}")
    ai, bi = np.isinf(a), np.isinf(b)
    if (ai != bi).any() or (ai & (np.sign(a) != np.sign(b))).any():
        k = np.flatnonzero((ai != bi) | (ai & (np.sign(a) != np.sign(b))))[:5]
        bad.append(f"{name}: inf mismatch: gpu={a[k]} ref={b[k]}")
    f = np.isfinite(a) & np.isfinite(b)
    err = np.abs(a[f] - b[f])
    lim = rtol * np.maximum(np.abs(a[f]), np.abs(b[f])) + atol
    if (err > lim).any():
        k = np.flatnonzero(err > lim)
        worst = k[np.argmax((err - lim)[k])]
        bad.append(f"{name}: {k.size} value mismatches; worst gpu={a[f][worst]!r} "
                   f"ref={b[f][worst]!r} err={err[worst]:.3e}")
    return bad
