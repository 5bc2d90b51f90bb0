"""Drop-in module name for the reference driver: `from MinuteFrequentFactorCICC import MinFreqFactor`."""
from mff.factor import MinFreqFactor  # noqa: F401
