"""stellard_amd -- MI355X-native batched Ed25519 transaction-signature
verification for stellard (hfeeki/stellard).

The hot path (SerializedTransaction::checkSign -> RippleAddress::verifySignature
-> crypto_sign_verify_detached) runs as hand-written gfx950 HIP kernels behind
the C ABI in include/stl.h (libstl.so).  This package is the Python mirror of
that boundary: see ``stellard_amd.verify`` and ``stellard_amd.protocol``.
"""
__version__ = "0.1.0"
