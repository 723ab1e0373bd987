"""parmmg_amd -- MI355X-native ParMmg post-remesh transfer path.

The product is ``libpmx_transfer.so`` (hand-written gfx950 HIP kernels behind the
C ABI of ``include/pmx_transfer.h``).  This package holds its ctypes binding
(:mod:`parmmg_amd._native`), the host-side mirror of the reference interface
(:mod:`parmmg_amd.transfer`) and the synthetic-input utilities
(:mod:`parmmg_amd.mesh`).
"""
from .mesh import Mesh  # noqa: F401

__all__ = ["Mesh"]
