"""h2o3_amd — an MI355X-native in-memory ML platform with H2O-3's capabilities.

Frames live in HBM as row-sharded torch tensors (one process per GPU,
RCCL/xGMI collectives across GPUs); the hot paths of the algorithms are
hand-written HIP kernels for gfx950 (see h2o3_amd/ops/csrc).
"""
__version__ = "0.1.0"

from .api import *  # noqa: F401,F403
from .api import H2OFrame  # noqa: F401
