"""jeromq_amd -- MI355X-native CurveZMQ MESSAGE crypto (JeroMQ CURVE per-message path).

  jeromq_amd.curve      Curve.java mirror: afternm / openAfternm (jnacl drop-ins)
  jeromq_amd.mechanism  CurveClientMechanism / CurveServerMechanism encode/decode (+ batches)
  jeromq_amd.batch      device-resident batched seal/open over torch tensors
  jeromq_amd._lib       ctypes binding of libcurvezmq_mi355x.so (include/curvezmq_mi355x.h)
"""
from . import _lib  # noqa: F401
from ._lib import CzError  # noqa: F401

__version__ = "0.1.0"
