"""CPU: the multi-day frame oracle (oracle_frame_xday) for the four factors whose
reference windows run over('code') only (CM:746, 862-867, 1216, 1238-1240) — it agrees
with the per-day oracle on a one-day frame and carries the cross-day terms on a two-day
frame, checked by hand."""
import numpy as np

import mff_oracle as O
from mff import synth


def test_frame_oracle_equals_per_day_oracle_on_one_day():
    panel = synth.make_panel(25, 1, config=31, ragged=True)
    ov, os_ = O.oracle_stage1(panel, O.FRAME_XDAY_NAMES)
    fx = O.oracle_frame_xday(panel)
    for i, nm in enumerate(O.FRAME_XDAY_NAMES):
        v, s = fx[nm]
        assert (s == os_[i]).all(), nm
        ok = s == O.VALUE
        np.testing.assert_allclose(v[ok], ov[i][ok], rtol=1e-12, atol=1e-15, equal_nan=True, err_msg=nm)


def _two_day_panel():
    """One code, two days, bars 0 and 225 present each day."""
    D, S = 2, 1
    p = {k: np.full((D, S, 240), np.nan, np.float32) for k in ("open", "high", "low", "close", "volume")}
    pres = np.zeros((D, S, 240), bool)
    for d, (c0, c1, v0, v1) in enumerate([(10.0, 10.5, 100.0, 200.0), (11.0, 10.0, 300.0, 400.0)]):
        for m, c, v in ((0, c0, v0), (225, c1, v1)):
            pres[d, 0, m] = True
            p["open"][d, 0, m] = 10.0
            p["high"][d, 0, m] = c
            p["low"][d, 0, m] = c
            p["close"][d, 0, m] = c
            p["volume"][d, 0, m] = v
    p["present"] = pres
    p["codes"] = ["000001.SZ"]
    p["dates"] = [0, 1]
    return p


def test_frame_oracle_cross_day_terms_by_hand():
    fx = O.oracle_frame_xday(_two_day_panel())
    am = fx["liq_amihud_1min"][0][:, 0]
    # day 0: bar 225 vs bar 0; day 1: bar 0 vs day 0's last close (10.5) -- the frame term
    assert am[0] == abs((10.5 - 10.0) / 10.0) / 200.0
    assert am[1] == abs((11.0 - 10.5) / 10.5) / 300.0 + abs((10.0 - 11.0) / 11.0) / 400.0
    b20 = fx["trade_bottom20retRatio"][0][:, 0]
    # 14:40+ rows: bar 225 of both days; volume_d over the whole frame: 200 + 400 + 1
    assert b20[0] == 200.0 / 601.0 * (10.5 / 10.0 - 1.0)
    assert b20[1] == 400.0 / 601.0 * (10.0 / 10.0 - 1.0)
    b50 = fx["trade_bottom50retRatio"][0][:, 0]
    assert b50[0] == 200.0 / 600.0 * (10.5 / 10.0 - 1.0)
    # corr_prvr: day 1 gets the cross-day pair -> two pairs (a constant-free pair set)
    pr_v, pr_s = fx["corr_prvr"]
    assert pr_s[0, 0] == O.VALUE and np.isnan(pr_v[0, 0])  # one pair on day 0: NaN (S3)
    assert pr_s[1, 0] == O.VALUE and abs(pr_v[1, 0] - 1.0) < 1e-12  # two pairs, both falling


def test_frame_doc_pdf_oracle_equals_per_day_on_one_day():
    """doc_pdf60..95 of a one-day frame: the frame-wide rank is the day's rank."""
    panel = synth.make_panel(25, 1, config=32, ragged=True)
    ov, os_ = O.oracle_stage1(panel, O.FRAME_RANK_NAMES)
    fx = O.oracle_frame_doc_pdf(panel)
    for i, nm in enumerate(O.FRAME_RANK_NAMES):
        v, s = fx[nm]
        assert (s == os_[i]).all(), nm
        assert (v == ov[i]).all(), nm


def test_frame_doc_pdf_ranks_every_date_by_hand():
    """CM:1015-1017 on a 2-day frame: `.rank()` is outside `.over`, so the four rows of
    both dates are ranked together.  Keys c_last/c: day 0 (10.5/10, 1.0), day 1
    (10/11, 1.0) -> frame ranks (4, 2.5), (1, 2.5); per day they would be (2, 1), (1, 2)."""
    fx = O.oracle_frame_xday(_two_day_panel())
    # day 0: levels rank 2.5 (share 2/3), rank 4 (share 1/3), cum-summed by ascending rank
    assert fx["doc_pdf60"][0][0, 0] == 2.5
    for nm in ("doc_pdf70", "doc_pdf80", "doc_pdf90", "doc_pdf95"):
        assert fx[nm][0][0, 0] == 4.0, nm
    # day 1: rank 1 (share 3/7), rank 2.5 (share 4/7): every threshold at rank 2.5
    for nm in O.FRAME_RANK_NAMES:
        assert fx[nm][0][1, 0] == 2.5 and fx[nm][1][1, 0] == O.VALUE, nm
    per_day = O.oracle_stage1(_two_day_panel(), ["doc_pdf60"])[0][0][:, 0]
    assert per_day.tolist() == [1.0, 2.0]
