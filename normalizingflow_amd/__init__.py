"""normalizingflow_amd -- MI355X-native coupling-layer hot path of
sherryli59/NormalizingFlow (flows' forward/inverse + log|det J| on HIP kernels).

Public surface mirrors the reference (re-exported as the ``nf`` package):
    from nf.flows import RealNVP, NSF_CL, NSF_AR, Planar, Radial, FCNN
    from nf.models import NormalizingFlowModel   # also NormalizingFlow
    from nf.utils import unconstrained_RQS, RQS, searchsorted
"""
from . import config  # noqa: F401
from ._lib import LIB_PATH, load as load_library  # noqa: F401
from .flows import FCNN, NSF_AR, NSF_CL, Planar, Radial, RealNVP  # noqa: F401
from .flows import MAF, ActNorm, OneByOneConv  # noqa: F401
from .flows import flush_status_checks  # noqa: F401
from .models import NormalizingFlow, NormalizingFlowModel  # noqa: F401

__version__ = "0.1.0"
