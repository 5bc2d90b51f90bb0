"""Test configuration: import paths and the `gpu` marker.

The product package lives in ``replication-of-minute-frequency-factor_amd/`` (not a valid
module name), so its directory is put on sys.path and imported as ``mff``; the oracle
directory is put on sys.path for the checker (tests only)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "replication-of-minute-frequency-factor_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs via gpurun)")
