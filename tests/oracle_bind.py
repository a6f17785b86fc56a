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


class TxInfo(ctypes.Structure):
    _fields_ = [("signing_len", ctypes.c_size_t), ("full_len", ctypes.c_size_t),
                ("pk_len", ctypes.c_long), ("sig_len", ctypes.c_long),
                ("pk", ctypes.c_uint8 * 64), ("sig", ctypes.c_uint8 * 64),
                ("max_depth", ctypes.c_int), ("all_declared", ctypes.c_int), ("stopped_early", ctypes.c_int)]


def pack_blobs(blobs):
    """(buffer, offsets u64, lengths u32) for a list of byte strings."""
    n = len(blobs)
    lens = np.array([len(b) for b in blobs], np.uint32)
    offs = np.zeros(n, np.uint64)
    if n:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(blobs) + b"\0" * 4, np.uint8).copy()
    return buf, offs, lens


class Oracle:
    def __init__(self, lib):
        self.lib = lib
        V = ctypes.c_void_p
        lib.oracle_verify.restype = ctypes.c_int
        lib.oracle_verify.argtypes = [V, V, ctypes.c_size_t, V, ctypes.c_uint32]
        lib.oracle_verify_raw.restype = ctypes.c_int
        lib.oracle_verify_raw.argtypes = [V, V, ctypes.c_size_t, V, ctypes.c_uint32]
        lib.oracle_verify_batch.argtypes = [V, V, V, ctypes.c_size_t, V, ctypes.c_uint32, ctypes.c_int]
        lib.oracle_tx_verify_batch.argtypes = [V, V, V, V, V, ctypes.c_size_t, V, ctypes.c_uint32, ctypes.c_int]
        lib.oracle_sha512.argtypes = [V, ctypes.c_size_t, V]
        lib.oracle_seed_keypair.argtypes = [V, V, V]
        lib.oracle_sign.argtypes = [V, V, ctypes.c_size_t, V]
        lib.oracle_tx_blob.restype = ctypes.c_int
        lib.oracle_tx_blob.argtypes = [V, ctypes.c_size_t, V, V, ctypes.c_size_t, ctypes.POINTER(TxInfo)]
        lib.oracle_tx_blob_verify_batch.argtypes = [V, V, V, ctypes.c_size_t, V, V, ctypes.c_uint32, ctypes.c_int]
        lib.oracle_signed_blob.restype = ctypes.c_int
        lib.oracle_signed_blob.argtypes = [ctypes.c_uint32, V, ctypes.c_size_t, V, V, ctypes.c_size_t,
                                           ctypes.POINTER(TxInfo)]
        lib.oracle_signed_blob_verify_batch.argtypes = [ctypes.c_uint32, V, V, V, ctypes.c_size_t, V, V,
                                                        ctypes.c_uint32, ctypes.c_int]

    def verify(self, sig, msg, pk, policy=0):
        return self.lib.oracle_verify(bytes(sig), bytes(msg), len(msg), bytes(pk), policy) == 0

    def verify_raw(self, sig, msg, pk, policy=0):
        """The bare crypto_sign_verify_detached predicate (no stellard S < L)."""
        return self.lib.oracle_verify_raw(bytes(sig), bytes(msg), len(msg), bytes(pk), policy) == 0

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

    def tx_blob(self, blob):
        """Reference re-serialisation of one blob: (ok, info, signing, full)."""
        cap = len(blob) + 64
        s = ctypes.create_string_buffer(cap)
        f = ctypes.create_string_buffer(cap)
        info = TxInfo()
        rc = self.lib.oracle_tx_blob(bytes(blob), len(blob), s, f, cap, ctypes.byref(info))
        return rc == 0, info, s.raw[:info.signing_len], f.raw[:info.full_len]

    def signed_blob(self, kind, blob):
        """Reference deserialise + re-serialise of one signed object (kind 0
        transaction, 1 validation): (ok, info, signing, full)."""
        cap = len(blob) + 64
        s = ctypes.create_string_buffer(cap)
        f = ctypes.create_string_buffer(cap)
        info = TxInfo()
        rc = self.lib.oracle_signed_blob(kind, bytes(blob), len(blob), s, f, cap, ctypes.byref(info))
        return rc == 0, info, s.raw[:info.signing_len], f.raw[:info.full_len]

    def signed_blob_verify_batch(self, kind, blobs, policy=0, threads=0, ids=False):
        buf, offs, lens = pack_blobs(blobs)
        n = len(blobs)
        bm = np.zeros((n + 7) // 8 or 1, np.uint8)
        idb = np.zeros((max(n, 1), 32), np.uint8)
        self.lib.oracle_signed_blob_verify_batch(kind, _buf(buf), _buf(offs), _buf(lens), n, _buf(bm),
                                                 _buf(idb) if ids else None, policy, threads)
        bits = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
        return (bits, idb[:n]) if ids else bits

    def tx_blob_verify_batch(self, blobs, policy=0, threads=0, tx_ids=False):
        buf, offs, lens = pack_blobs(blobs)
        n = len(blobs)
        bm = np.zeros((n + 7) // 8 or 1, np.uint8)
        ids = np.zeros((max(n, 1), 32), np.uint8)
        self.lib.oracle_tx_blob_verify_batch(_buf(buf), _buf(offs), _buf(lens), n, _buf(bm),
                                             _buf(ids) if tx_ids else None, policy, threads)
        bits = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
        return (bits, ids[:n]) if tx_ids else bits


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
    lib.ref_tx_blob_verify_batch.argtypes = [V, V, V, ctypes.c_size_t, V, V, ctypes.c_uint32, ctypes.c_int]
    lib.ref_sign_batch.argtypes = [V, V, ctypes.c_size_t, V, V, ctypes.c_int]
    lib.ref_signed_blob_verify_batch.argtypes = [ctypes.c_uint32, V, V, V, ctypes.c_size_t, V, V, ctypes.c_uint32,
                                                 ctypes.c_int]
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


def sodium_tx_blob_verify_batch(lib, blobs, threads=0, tx_ids=False):
    buf, offs, lens = pack_blobs(blobs)
    n = len(blobs)
    bm = np.zeros((n + 7) // 8 or 1, np.uint8)
    ids = np.zeros((max(n, 1), 32), np.uint8)
    lib.ref_tx_blob_verify_batch(_buf(buf), _buf(offs), _buf(lens), n, _buf(bm), _buf(ids) if tx_ids else None,
                                 0, threads)
    bits = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
    return (bits, ids[:n]) if tx_ids else bits


def sodium_sign_batch(lib, seeds, msgs, threads=0):
    """libsodium keypair(seed_i) + detached signature over msg_i (32 B)."""
    seeds = np.ascontiguousarray(seeds, np.uint8)
    msgs = np.ascontiguousarray(msgs, np.uint8)
    n = seeds.shape[0]
    pk = np.empty((n, 32), np.uint8)
    sig = np.empty((n, 64), np.uint8)
    lib.ref_sign_batch(_buf(seeds), _buf(msgs), n, _buf(pk), _buf(sig), threads)
    return pk, sig


def sodium_signed_blob_verify_batch(lib, kind, blobs, threads=0, ids=False):
    buf, offs, lens = pack_blobs(blobs)
    n = len(blobs)
    bm = np.zeros((n + 7) // 8 or 1, np.uint8)
    idb = np.zeros((max(n, 1), 32), np.uint8)
    lib.ref_signed_blob_verify_batch(kind, _buf(buf), _buf(offs), _buf(lens), n, _buf(bm),
                                     _buf(idb) if ids else None, 0, threads)
    bits = np.unpackbits(bm, bitorder="little")[:n].astype(bool)
    return (bits, idb[:n]) if ids else bits


def hostemu_signed_blob(lib, kind, blob):
    """Device pass (either kind) compiled for the host: (status, msg, id)."""
    st = ctypes.c_uint32(0)
    msg = ctypes.create_string_buffer(32)
    idb = ctypes.create_string_buffer(32)
    arr = np.frombuffer(bytes(blob) + b"\0" * 4, np.uint8).copy()
    lib.hostemu_signed_blob(kind, _buf(arr), len(blob), ctypes.byref(st), msg, idb)
    return st.value, msg.raw, idb.raw


def hostemu_sign_adversarial(lib, seeds, msgs, cls, param):
    """stl_sign.h compiled for the host: (pk, sig, msg) of the rows the GPU's
    sign kernel builds."""
    n = seeds.shape[0]
    seeds, msgs = np.ascontiguousarray(seeds, np.uint8), np.ascontiguousarray(msgs, np.uint8)
    cls, param = np.ascontiguousarray(cls, np.uint8), np.ascontiguousarray(param, np.uint32)
    pk = np.empty((n, 32), np.uint8)
    sig = np.empty((n, 64), np.uint8)
    mo = np.empty((n, 32), np.uint8)
    lib.hostemu_sign_adversarial(_buf(seeds), _buf(msgs), _buf(cls), _buf(param), n, _buf(pk), _buf(sig), _buf(mo))
    return pk, sig, mo


def hostemu_tx_blob(lib, blob):
    """Device pass compiled for the host: (status, msg, txid, layout)."""
    st = ctypes.c_uint32(0)
    msg = ctypes.create_string_buffer(32)
    tid = ctypes.create_string_buffer(32)
    lay = (ctypes.c_uint32 * 10)()
    b = bytes(blob) + b"\0" * 4
    arr = np.frombuffer(b, np.uint8).copy()
    lib.hostemu_tx_blob(_buf(arr), len(blob), ctypes.byref(st), msg, tid, lay)
    return st.value, msg.raw, tid.raw, list(lay)


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
    lib.hostemu_verify_batch_split.restype = ctypes.c_uint64
    lib.hostemu_verify_batch_split.argtypes = [V, V, V, ctypes.c_size_t, V, ctypes.c_uint32, ctypes.c_int]
    lib.hostemu_verify_batch_joint.restype = ctypes.c_uint64
    lib.hostemu_verify_batch_joint.argtypes = [V, V, V, ctypes.c_size_t, V, ctypes.c_uint32, ctypes.c_int]
    lib.hostemu_verify_batch_pair.restype = ctypes.c_uint64
    lib.hostemu_verify_batch_pair.argtypes = [V, V, V, ctypes.c_size_t, V, ctypes.c_uint32]
    lib.hostemu_identity_head.argtypes = [V]
    lib.hostemu_lattice.restype = ctypes.c_int
    lib.hostemu_lattice.argtypes = [V, V, V, V]
    lib.hostemu_sc_mul_signed.argtypes = [V, ctypes.c_int, V, V]
    lib.hostemu_sha512_half.argtypes = [V, ctypes.c_uint32, V]
    lib.hostemu_sha512_pair_compress.argtypes = [V, V, ctypes.c_int]
    lib.hostemu_tx_blob.argtypes = [V, ctypes.c_uint32, V, V, V, V]
    lib.hostemu_signed_blob.argtypes = [ctypes.c_uint32, V, ctypes.c_uint32, V, V, V]
    lib.hostemu_blob_words.argtypes = [V, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, V]
    lib.hostemu_wide_row.argtypes = [ctypes.c_int, ctypes.c_uint32, V]
    lib.hostemu_wide_key_table.restype = ctypes.c_int
    lib.hostemu_wide_key_table.argtypes = [V, V, V]
    lib.hostemu_sign_adversarial.argtypes = [V, V, V, V, ctypes.c_size_t, V, V, V]
    lib.hostemu_window_blocks.restype = ctypes.c_uint32
    lib.hostemu_window_blocks.argtypes = [V, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int]
    return lib
