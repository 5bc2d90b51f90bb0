"""Drop-in module name for the reference's factor file: `import MinuteFrequentFactorCalculateMethodsCICC`
gives the 58 `cal_*` functions, each running on the MI355X stage-1 kernel (see mff.factors)."""
from mff.factors import *  # noqa: F401,F403
from mff.factors import __all__  # noqa: F401
