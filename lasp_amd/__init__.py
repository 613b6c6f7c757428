"""lasp_amd — MI355X-native batched lattice-join engine for Lasp's CRDT hot path.

Product layers (no CPU fallback anywhere; a missing HIP library raises
LaspjUnavailable):
  csrc/        HIP kernels for gfx950 + the C ABI (include/laspj.h) -> liblaspj.so
  _lib         ctypes binding of the C ABI (stand-in for the Erlang NIF)
  engine       device-resident OR-Set / G-Set batches (Context, ORSetBatch, GSetBatch)
  terms/codec  Erlang term order + orddict <-> columnar dictionaries
  orset/gset/lattice/core   mirrors of lasp_orset / lasp_gset / lasp_lattice /
               lasp_core over the engine
"""

from ._lib import LaspjError, LaspjUnavailable  # noqa: F401

__all__ = ["LaspjError", "LaspjUnavailable"]
