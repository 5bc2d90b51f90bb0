"""Drop-in module name for the reference base class: `from Factor import Factor`."""
from mff.factor import Factor  # noqa: F401
