"""``nf.flows_1`` of the reference: Planar / Radial / MAF / ActNorm / OneByOneConv (and the shared layers)."""
from normalizingflow_amd.flows import FCNN, NSF_CL, Planar, Radial, RealNVP  # noqa: F401
from normalizingflow_amd.flows import MAF, ActNorm, NSF_AR, OneByOneConv  # noqa: F401
from normalizingflow_amd.flows import functional_derivatives  # noqa: F401
