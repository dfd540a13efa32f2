"""``nf.flows`` of the reference (nf/flows.py, nf/flows_1.py): same names, HIP-backed."""
from normalizingflow_amd.flows import *  # noqa: F401,F403
from normalizingflow_amd.flows import FCNN, NSF_AR, NSF_CL, Planar, Radial, RealNVP  # noqa: F401
from normalizingflow_amd.flows import functional_derivatives  # noqa: F401
