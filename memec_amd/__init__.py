"""memec_amd — MI355X-native erasure-coding engine for MemEC's stripe
encode/decode path (RS and Cauchy-RS), behind MemEC's common/coding plugin
surface.

Layers:
  include/mec.h            C ABI (libmec.so, memec_amd/csrc/*.hip, *.cpp)
  memec_amd/csrc/coding/   C++ drop-in for class Coding (libmemec_coding.so)
  memec_amd.codec          Python binding of the C ABI (tests, bench)
"""
from ._lib import FAMILIES, MecError, lib, set_knob  # noqa: F401
from .codec import Codec, fill_random, host_register, host_unregister, xor  # noqa: F401

__all__ = ["Codec", "MecError", "FAMILIES", "fill_random", "xor", "host_register", "host_unregister", "lib", "set_knob"]
