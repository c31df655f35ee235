"""narwhal_amd — MI355X-native Ed25519 verify + SHA-512 digest engine for Narwhal/Bullshark.

Drop-in for the reference ``crypto`` crate's hot path:
``narwhal_amd.crypto`` mirrors crypto/src/lib.rs; ``narwhal_amd.shard`` is the multi-GPU
sharding layer; ``narwhal_amd.workload`` builds the synthetic committees and certificates.
All compute runs in libnwcrypto.so (hand-written gfx950 HIP); importing without the built
library raises ImportError.
"""
from . import _lib  # noqa: F401  (fails loudly when libnwcrypto.so is missing)
from ._lib import DeviceError, Engine, default_engine, version  # noqa: F401

__all__ = ["Engine", "DeviceError", "default_engine", "version"]
