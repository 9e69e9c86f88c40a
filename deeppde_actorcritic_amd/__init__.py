"""deeppde_actorcritic_amd — MI355X-native hot path of the actor-critic HJB solver.

Drop-in for MoZhou1995/DeepPDE_ActorCritic's `equation` / `solver` modules:
the batched boundary-stopped SDE rollout, running-cost accumulation and
VR-LSTD / LSTD target assembly run as HIP kernels for gfx950 (libdpac.so,
C ABI in include/dpac.h), as do the MLPs (MFMA kernels, fused into the actor's
rollout and BPTT), their parameter gradients and the Adam update; PyTorch-ROCm
provides device memory, streams, HIP graphs and torch.distributed (RCCL).
"""
from . import _lib, config, equation, ops, parallel, solver  # noqa: F401
from .config import load_config, munchify, set_floatx  # noqa: F401
from .equation import EKN, LQR, LQR_var, VDP, Equation, TrajectoryBatch, ekn  # noqa: F401
from .solver import ActorCriticSolver, ActorModel, CriticModel, DeepNN  # noqa: F401

__version__ = "0.1.0"
