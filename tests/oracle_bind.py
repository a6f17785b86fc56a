"""ctypes bindings of the test-only checkers under oracle/ (never imported by
the product package).  Builds them on first use if the .so files are absent
and a compiler is available."""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "liboracle.so")
SODIUM_REF_SO = os.path.join(ROOT, "oracle", "_ref", "libsodium_ref.so")
HOSTEMU_SO = os.path.join(ROOT, "tests", "native", "libhostemu.so")


def _buf(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class Oracle:
    def __init__(self, lib):
        self.lib = lib
        V = ctypes.c_void_p
        lib.oracle_verify.restype = ctypes.c_int
        lib.oracle_verify.argtypes = [V, V, ctypes.c_size_t, V, ctypes.c_uint32]
        lib.oracle_verify_batch.argtypes = [V, V, V, ctypes.c_size_t, V, ctypes.c_uint32, ctypes.c_int]
        lib.oracle_tx_verify_batch.argtypes = [V, V, V, V, V, ctypes.c_size_t, V, ctypes.c_uint32, ctypes.c_int]
        lib.oracle_sha512.argtypes = [V, ctypes.c_size_t, V]
        lib.oracle_seed_keypair.argtypes = [V, V, V]
        lib.oracle_sign.argtypes = [V, V, ctypes.c_size_t, V]

    def verify(self, sig, msg, pk, policy=0):
        return self.lib.oracle_verify(bytes(sig), bytes(msg), len(msg), bytes(pk), policy) == 0

    def verify_batch(self, sig, msg, pk, policy=0, threads=0):
        sig = np.ascontiguousarray(sig, np.uint8)
        msg = np.ascontiguousarray(msg, np.uint8)
        pk = np.ascontiguousarray(pk, np.uint8)
        n = sig.shape[0]
        bm = np.zeros((n + 7) // 8, np.uint8)
        self.lib.oracle_verify_batch(_buf(sig), _buf(msg), _buf(pk), n, _buf(bm), policy, threads)
        return np.unpackbits(bm, bitorder="little")[:n].astype(bool)

    def tx_verify_batch(self, preimages, sig, pk, policy=0, threads=0):
        n = len(preimages)
        lens = np.array([len(p) for p in preimages], np.uint32)
        offs = np.zeros(n, np.uint64)
        if n:
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        blob = np.frombuffer(b"".join(preimages) or b"\0", np.uint8).copy()
        sig = np.ascontiguousarray(sig, np.uint8)
        pk = np.ascontiguousarray(pk, np.uint8)
        bm = np.zeros((n + 7) // 8, np.uint8)
        self.lib.oracle_tx_verify_batch(_buf(blob), _buf(offs), _buf(lens), _buf(sig), _buf(pk), n, _buf(bm),
                                        policy, threads)
        return np.unpackbits(bm, bitorder="little")[:n].astype(bool)

    def keypair(self, seed):
        pk = ctypes.create_string_buffer(32)
        sk = ctypes.create_string_buffer(64)
        self.lib.oracle_seed_keypair(pk, sk, bytes(seed))
        return pk.raw, sk.raw

    def sign(self, msg, sk):
        sig = ctypes.create_string_buffer(64)
        self.lib.oracle_sign(sig, bytes(msg), len(msg), bytes(sk))
        return sig.raw

    def sha512(self, data):
        out = ctypes.create_string_buffer(64)
        self.lib.oracle_sha512(bytes(data), len(data), out)
        return out.raw


def _ensure(path, target):
    if not os.path.exists(path):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), target], check=True)


def load_oracle():
    _ensure(ORACLE_SO, "build/liboracle.so")
    return Oracle(ctypes.CDLL(ORACLE_SO))


def load_sodium_ref():
    """The reference's verify call path over libsodium 1.0.18 + OpenSSL, or None
    where libsodium is absent."""
    if not os.path.exists(SODIUM_REF_SO):
        if not os.path.exists("/opt/conda/include/sodium.h"):
            return None
        _ensure(SODIUM_REF_SO, "_ref/libsodium_ref.so")
    try:
        lib = ctypes.CDLL(SODIUM_REF_SO)
    except OSError:
        return None
    V = ctypes.c_void_p
    lib.ref_init.restype = ctypes.c_int
    lib.ref_sodium_version.restype = ctypes.c_char_p
    lib.ref_verify_batch.argtypes = [V, V, V, ctypes.c_size_t, V, ctypes.c_int]
    lib.ref_tx_verify_batch.argtypes = [V, V, V, V, V, ctypes.c_size_t, V, ctypes.c_int]
    lib.ref_verify_signature.argtypes = [V, V, V]
    lib.ref_crypto_sign_verify_detached.argtypes = [V, V, ctypes.c_ulonglong, V]
    lib.ref_seed_keypair.argtypes = [V, V, V]
    lib.ref_sign_detached.argtypes = [V, V, ctypes.c_ulonglong, V]
    if lib.ref_init() != 0:
        return None
    return lib


def sodium_verify_batch(lib, sig, msg, pk, threads=0):
    sig = np.ascontiguousarray(sig, np.uint8)
    msg = np.ascontiguousarray(msg, np.uint8)
    pk = np.ascontiguousarray(pk, np.uint8)
    n = sig.shape[0]
    bm = np.zeros((n + 7) // 8, np.uint8)
    lib.ref_verify_batch(_buf(sig), _buf(msg), _buf(pk), n, _buf(bm), threads)
    return np.unpackbits(bm, bitorder="little")[:n].astype(bool)


def load_hostemu():
    if not os.path.exists(HOSTEMU_SO):
        from stellard_amd import build
        build.build_hostemu()
    lib = ctypes.CDLL(HOSTEMU_SO)
    V = ctypes.c_void_p
    lib.hostemu_verify_batch.restype = ctypes.c_uint64
    lib.hostemu_verify_batch.argtypes = [V, V, V, ctypes.c_size_t, V, ctypes.c_uint32]
    lib.hostemu_bound_checks.restype = ctypes.c_uint64
    lib.hostemu_verify_batch_mode.restype = ctypes.c_uint64
    lib.hostemu_verify_batch_mode.argtypes = [V, V, V, ctypes.c_size_t, V, ctypes.c_uint32, ctypes.c_int, V]
    lib.hostemu_lattice.restype = ctypes.c_int
    lib.hostemu_lattice.argtypes = [V, V, V, V]
    lib.hostemu_sc_mul_signed.argtypes = [V, ctypes.c_int, V, V]
    lib.hostemu_sha512_half.argtypes = [V, ctypes.c_uint32, V]
    return lib
