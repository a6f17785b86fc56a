"""stellard_amd -- MI355X-native batched Ed25519 transaction-signature
verification for stellard (hfeeki/stellard).

The hot path (SerializedTransaction::checkSign -> RippleAddress::verifySignature
-> crypto_sign_verify_detached) runs as hand-written gfx950 HIP kernels behind
the C ABI in include/stl.h (libstl.so).  This package is the Python mirror of
that boundary: ``stellard_amd.verify`` (the reference's verify / checkSign
calls, the aggregator, the multi-GPU communicator), ``stellard_amd.shard``
(index and byte shards, gloo-side gathers) and ``stellard_amd._native`` (the
ctypes binding of every symbol stl.h declares).
"""
__version__ = "0.2.0"
