"""``nf.utils`` of the reference (nf/utils.py): spline functions, HIP-backed."""
from normalizingflow_amd.utils import *  # noqa: F401,F403
from normalizingflow_amd.utils import RQS, searchsorted, unconstrained_RQS  # noqa: F401
