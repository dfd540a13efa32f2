"""``nf.flows_1`` of the reference: its own NSF_AR (flows_1.py:395-465) and the shared layers."""
from normalizingflow_amd.flows_1 import *  # noqa: F401,F403
from normalizingflow_amd.flows_1 import (NSF_AR, NSF_CL, ActNorm, FCNN, MAF, OneByOneConv,  # noqa: F401
                                         Planar, Radial, RealNVP, functional_derivatives)
