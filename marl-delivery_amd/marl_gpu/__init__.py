"""marl_gpu -- MI355X-native batched step engine for the marl-delivery grid world.

Host side of the engine: a ctypes binding of the C ABI (include/mdl_engine.h),
the tensor API (``BatchedEnv``), and drop-in shims of the reference's dict API
(``compat.Environment`` / ``compat.VectorizedEnv``) and helper functions
(``helper``).  All env transitions and observation builders run as gfx950 HIP
kernels in ``libmdl.so``; there is no CPU execution path.
"""
from ._lib import MdlError, lib
from .engine import MAPPO_SHAPING, QMIX_SHAPING, BatchedEnv

__all__ = ["BatchedEnv", "MdlError", "MAPPO_SHAPING", "QMIX_SHAPING", "lib"]
__version__ = "0.1.0"
