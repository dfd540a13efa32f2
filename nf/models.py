"""``nf.models`` of the reference (nf/models.py)."""
from normalizingflow_amd.models import NormalizingFlow, NormalizingFlowModel  # noqa: F401
