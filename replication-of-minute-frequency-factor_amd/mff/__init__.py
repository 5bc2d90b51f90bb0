"""mff — MI355X-native CICC minute-frequency factor engine.

Host-side mirror of the reference interface (C-X-Lu/Replication-of-Minute-Frequency-Factor)
over libmff.so (hand-written HIP for gfx950):

* :mod:`mff.factors`  — the 58 ``cal_*`` drop-in functions (MinuteFrequentFactorCalculateMethodsCICC.py)
* :mod:`mff.factor`   — ``Factor`` / ``MinFreqFactor`` (Factor.py, MinuteFrequentFactorCICC.py)
* :mod:`mff.engine`   — dense-panel device API (stage 1 / 2 / 3)
* :mod:`mff.dist`     — one process per GPU, stock-sharded, RCCL collectives
"""
from . import catalog  # noqa: F401

__version__ = "0.1.0"
