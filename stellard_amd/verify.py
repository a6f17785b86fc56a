"""Python mirror of stellard's signature-check interface over libstl.

Reference interface being mirrored (hfeeki/stellard):
  * RippleAddress::verifySignature(uint256 const&, Blob const&)
      src/ripple_data/protocol/RippleAddress.cpp:190-200
      -> throws std::runtime_error("bad inputs to verifySignature") when the
         key is not 32 bytes or the signature not 64 bytes (:192-194);
         returns crypto_sign_verify_detached(...) == 0 && S < L.
  * StellarPublicKey::verifySignature  src/ripple_data/crypto/StellarPublicKey.cpp:67-77
  * SerializedTransaction::checkSign(const RippleAddress&)
      src/ripple_app/misc/SerializedTransaction.cpp:220-230 (any exception -> false)

Every call goes to the gfx950 kernels through the C ABI; nothing here
verifies on the CPU.
"""
import ctypes

import numpy as np

from . import _native as N

POLICY_SODIUM_1_0_18 = N.STL_POLICY_SODIUM_1_0_18
POLICY_STELLARD_1_0_0 = N.STL_POLICY_STELLARD_1_0_0
# OR into `policy` to check with full-length scalars (same bits, slower)
FULL_LENGTH = N.STL_FULL_LENGTH
# OR into `policy` to decode each distinct public key of a batch once
DEDUP_KEYS = N.STL_DEDUP_KEYS
ONE_LANE = N.STL_ONE_LANE
NO_AUTO_DEDUP = N.STL_NO_AUTO_DEDUP


class BadInputs(RuntimeError):
    """std::runtime_error("bad inputs to verifySignature") (RippleAddress.cpp:193)."""


def _buf(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# libsodium's crypto_sign_verify_detached signature (stl_verify_fn)
VERIFY_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_ulonglong, ctypes.c_void_p)


class Config(ctypes.Structure):
    """stl_config (include/stl.h, ABI 3)."""
    _fields_ = [("struct_size", ctypes.c_uint32), ("device_count", ctypes.c_int32),
                ("first_device", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("shards_per_device", ctypes.c_int32), ("reserved", ctypes.c_uint32),
                ("fallback_verify", VERIFY_FN)]


_fallback_keepalive = []


def init(device_count=0, first_device=0, flags=0, shards_per_device=1, fallback_verify=None):
    """stl_init (sodium_init's place, ripple_app.cpp:129-132).  flags:
    N.STL_CFG_RCCL_GATHER / N.STL_CFG_NO_RCCL.  ``fallback_verify``: a
    VERIFY_FN (the caller's libsodium check) that stl_ed25519_verify_detached
    answers device failures with."""
    fb = fallback_verify if fallback_verify is not None else VERIFY_FN()
    if fallback_verify is not None:
        _fallback_keepalive.append(fallback_verify)  # libstl keeps the pointer
    cfg = Config(ctypes.sizeof(Config), device_count, first_device, flags, shards_per_device, 0, fb)
    return N.check(N.load().stl_init(ctypes.byref(cfg)), "stl_init")


def shutdown():
    N.load().stl_shutdown()


def shard_range(n, rank, world):
    """stl_shard_range: contiguous 64-aligned index shard of rank r."""
    lo, hi = ctypes.c_size_t(0), ctypes.c_size_t(0)
    N.load().stl_shard_range(n, rank, world, ctypes.byref(lo), ctypes.byref(hi))
    return lo.value, hi.value


def shard_range_bytes(lens, rank, world):
    """stl_shard_range_bytes: byte-balanced 64-aligned shard of rank r."""
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    lo, hi = ctypes.c_size_t(0), ctypes.c_size_t(0)
    N.load().stl_shard_range_bytes(_buf(lens), lens.shape[0], rank, world, ctypes.byref(lo), ctypes.byref(hi))
    return lo.value, hi.value


def verify_signature(hash32, sig, pk):
    """RippleAddress::verifySignature: bool, raises BadInputs on size mismatch."""
    pk, sig, hash32 = bytes(pk), bytes(sig), bytes(hash32)
    if len(pk) != 32 or len(sig) != 64:
        raise BadInputs("bad inputs to verifySignature")
    rc = N.load().stl_ed25519_verify_detached(sig, hash32, len(hash32), pk)
    if rc == 0:
        return True
    if rc == -1:
        return False
    raise N.StlError(rc, "stl_ed25519_verify_detached")


def crypto_sign_verify_detached(sig, m, pk):
    """libsodium call surface: 0 accept / -1 reject (+ stellard's S<L)."""
    sig, m, pk = bytes(sig), bytes(m), bytes(pk)
    if len(sig) != 64 or len(pk) != 32:
        return -1
    rc = N.load().stl_ed25519_verify_detached(sig, m, len(m), pk)
    if rc in (0, -1):
        return rc
    raise N.StlError(rc, "stl_ed25519_verify_detached")


def unpack_bitmap(bitmap, n):
    return np.unpackbits(np.frombuffer(bytes(bitmap), dtype=np.uint8), bitorder="little")[:n].astype(bool)


def verify_batch(sig, msg, pk, policy=POLICY_SODIUM_1_0_18):
    """Batch RippleAddress::verifySignature over host arrays -> bool[n]."""
    sig = np.ascontiguousarray(sig, dtype=np.uint8).reshape(-1, 64)
    msg = np.ascontiguousarray(msg, dtype=np.uint8).reshape(-1, 32)
    pk = np.ascontiguousarray(pk, dtype=np.uint8).reshape(-1, 32)
    n = sig.shape[0]
    if msg.shape[0] != n or pk.shape[0] != n:
        raise ValueError("sig/msg/pk batch sizes differ")
    bitmap = np.zeros((n + 7) // 8, dtype=np.uint8)
    N.check(N.load().stl_ed25519_verify_batch(_buf(sig), _buf(msg), _buf(pk), n, _buf(bitmap), policy),
            "stl_ed25519_verify_batch")
    return unpack_bitmap(bitmap, n)


def tx_verify_batch(preimages, sig, pk, policy=POLICY_SODIUM_1_0_18):
    """Batch checkSign: preimages is a list of bytes ("STX\\0" || fields)."""
    n = len(preimages)
    lens = np.array([len(p) for p in preimages], dtype=np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    if n:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    blob = np.frombuffer(b"".join(bytes(p) for p in preimages) or b"\0", dtype=np.uint8).copy()
    sig = np.ascontiguousarray(sig, dtype=np.uint8).reshape(-1, 64)
    pk = np.ascontiguousarray(pk, dtype=np.uint8).reshape(-1, 32)
    bitmap = np.zeros((n + 7) // 8, dtype=np.uint8)
    N.check(N.load().stl_tx_verify_batch(_buf(blob), _buf(offs), _buf(lens), _buf(sig), _buf(pk), n,
                                         _buf(bitmap), policy), "stl_tx_verify_batch")
    return unpack_bitmap(bitmap, n)


def _pack(chunks):
    n = len(chunks)
    lens = np.array([len(p) for p in chunks], dtype=np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    if n:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(bytes(p) for p in chunks) + b"\0" * 4, dtype=np.uint8).copy()
    return buf, offs, lens


TX_OK, TX_DEFERRED, TX_MALFORMED = N.STL_TX_OK, N.STL_TX_DEFERRED, N.STL_TX_MALFORMED


BLOB_TRANSACTION, BLOB_VALIDATION = N.STL_BLOB_TRANSACTION, N.STL_BLOB_VALIDATION


def signed_blob_verify_batch(blobs, kind=BLOB_TRANSACTION, policy=POLICY_SODIUM_1_0_18, ids=False):
    """stl_signed_blob_verify_batch: the signature check of serialized signed
    objects (list of bytes).  kind BLOB_TRANSACTION = checkSign,
    BLOB_VALIDATION = SerializedValidation::isValid.  Returns (accept bool[n],
    status uint8[n]) plus the IDs (n, 32) when ``ids``."""
    n = len(blobs)
    buf, offs, lens = _pack(blobs)
    bitmap = np.zeros((n + 7) // 8 or 1, dtype=np.uint8)
    status = np.zeros(max(n, 1), dtype=np.uint8)
    idb = np.zeros((max(n, 1), 32), dtype=np.uint8) if ids else None
    N.check(N.load().stl_signed_blob_verify_batch(kind, _buf(buf), _buf(offs), _buf(lens), n, _buf(bitmap),
                                                  _buf(status), _buf(idb) if ids else None, policy),
            "stl_signed_blob_verify_batch")
    bits = unpack_bitmap(bitmap, n)
    return (bits, status[:n], idb[:n]) if ids else (bits, status[:n])


def tx_blob_verify_batch(blobs, policy=POLICY_SODIUM_1_0_18, tx_ids=False):
    """checkSign straight from serialized transactions (list of bytes, each
    the whole transaction with its TxnSignature).  Returns (accept bool[n],
    status uint8[n]) -- status TX_OK / TX_DEFERRED / TX_MALFORMED, see
    include/stl.h -- plus the transaction IDs (n, 32) when ``tx_ids``."""
    n = len(blobs)
    buf, offs, lens = _pack(blobs)
    bitmap = np.zeros((n + 7) // 8 or 1, dtype=np.uint8)
    status = np.zeros(max(n, 1), dtype=np.uint8)
    ids = np.zeros((max(n, 1), 32), dtype=np.uint8) if tx_ids else None
    N.check(N.load().stl_tx_blob_verify_batch(_buf(buf), _buf(offs), _buf(lens), n, _buf(bitmap), _buf(status),
                                              _buf(ids) if tx_ids else None, policy), "stl_tx_blob_verify_batch")
    bits = unpack_bitmap(bitmap, n)
    return (bits, status[:n], ids[:n]) if tx_ids else (bits, status[:n])


def proposal_preimage(propose_seq, close_time, prev_ledger, position):
    """LedgerProposal::getSigningHash preimage (LedgerProposal.cpp:54-65):
    "PRP\0" || seq || closeTime (big-endian u32, Serializer::add32) ||
    previous ledger || position (uint256 bytes, add256); 76 bytes."""
    prev_ledger, position = bytes(prev_ledger), bytes(position)
    if len(prev_ledger) != 32 or len(position) != 32:
        raise ValueError("ledger hashes are 32 bytes")
    return (b"PRP\x00" + int(propose_seq).to_bytes(4, "big") + int(close_time).to_bytes(4, "big")
            + prev_ledger + position)


# ---- transaction level: SerializedTransaction::checkSign ----

class SignedTx:
    """The signature-check state of one SerializedTransaction.

    Mirrors src/ripple_app/misc/SerializedTransaction.cpp:192-230 and the
    cache flags of SerializedTransaction.h:116-131: ``signing_pub_key`` is the
    sfSigningPubKey VL field (any length), ``txn_signature`` the sfTxnSignature
    VL field (None when absent: getFieldVL returns an empty Blob,
    SerializedObject.cpp:814), ``preimage`` the signing preimage
    "STX\\0" || fields without TxnSignature (STObject::getSigningHash,
    SerializedObject.cpp:444-450)."""

    def __init__(self, signing_pub_key, txn_signature, preimage):
        self.signing_pub_key = bytes(signing_pub_key)
        self.txn_signature = None if txn_signature is None else bytes(txn_signature)
        self.preimage = bytes(preimage)
        self.sig_good = False   # mSigGood
        self.sig_bad = False    # mSigBad

    def well_formed(self):
        """verifySignature throws on a key that is not 32 bytes or a signature
        that is not 64 (RippleAddress.cpp:192-194); checkSign maps the throw to
        false (SerializedTransaction.cpp:211-217, 226-229)."""
        return len(self.signing_pub_key) == 32 and self.txn_signature is not None and len(self.txn_signature) == 64

    def set_good(self):
        self.sig_good = True

    def check_sign(self, policy=POLICY_SODIUM_1_0_18):
        """SerializedTransaction::checkSign(): cached verdict, else verify."""
        return check_sign_batch([self], policy=policy)[0]


def check_sign_batch(txs, policy=POLICY_SODIUM_1_0_18, mark="both"):
    """checkSign over many transactions with one stl_tx_verify_batch call.

    Cached rows return their verdict (mSigGood / mSigBad); malformed rows are
    rejected on the host and never reach the GPU.  ``mark="both"`` records
    both verdicts like the serial path; ``mark="good_only"`` records accepts
    only -- the ledger-close pre-verify, which must
    not call setBad() because LedgerConsensus.cpp:2101-2106 applies unflagged
    transactions without a signature check.  Returns a list of bools."""
    if mark not in ("both", "good_only"):
        raise ValueError("mark must be 'both' or 'good_only'")
    out = [False] * len(txs)
    todo = []
    for i, t in enumerate(txs):
        if t.sig_good:
            out[i] = True
        elif t.sig_bad:
            out[i] = False
        elif not t.well_formed():
            if mark == "both":
                t.sig_bad = True
        else:
            todo.append(i)
    if todo:
        sig = np.frombuffer(b"".join(txs[i].txn_signature for i in todo), np.uint8).reshape(-1, 64)
        pk = np.frombuffer(b"".join(txs[i].signing_pub_key for i in todo), np.uint8).reshape(-1, 32)
        bits = tx_verify_batch([txs[i].preimage for i in todo], sig, pk, policy=policy)
        for i, b in zip(todo, bits):
            out[i] = bool(b)
            if b:
                txs[i].sig_good = True
            elif mark == "both":
                txs[i].sig_bad = True
    return out


# ---- device-resident (torch tensors as HBM buffers; torch is plumbing only) ----

def _stream_ptr(stream):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def verify_batch_device(sig, msg, pk, out_words=None, policy=POLICY_SODIUM_1_0_18, stream=None):
    """sig (n,64) / msg (n,32) / pk (n,32) uint8 CUDA tensors -> int64[ceil(n/64)]
    bitmap words (async on ``stream``)."""
    import torch
    n = sig.shape[0]
    if out_words is None:
        out_words = torch.empty((n + 63) // 64, dtype=torch.int64, device=sig.device)
    for t in (sig, msg, pk, out_words):
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("device entry point needs contiguous CUDA tensors")
    N.check(N.load().stl_ed25519_verify_batch_device(
        ctypes.c_void_p(sig.data_ptr()), ctypes.c_void_p(msg.data_ptr()), ctypes.c_void_p(pk.data_ptr()), n,
        ctypes.c_void_p(out_words.data_ptr()), policy, _stream_ptr(stream)), "stl_ed25519_verify_batch_device")
    return out_words


def tx_hash_batch_device(preimages, offsets, lengths, out_msg=None, stream=None):
    """SHA512Half of signing preimages already in HBM (uint8 / int64 / int32
    CUDA tensors; getSigningHash, SerializedObject.cpp:444-450) -> (n,32) uint8
    signing hashes, asynchronously on ``stream``; with verify_batch_device this
    is the device-resident checkSign (stl_tx_verify_batch)."""
    import torch
    n = offsets.shape[0]
    if out_msg is None:
        out_msg = torch.empty((n, 32), dtype=torch.uint8, device=preimages.device)
    for t in (preimages, offsets, lengths, out_msg):
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("device entry point needs contiguous CUDA tensors")
    if offsets.dtype != torch.int64 or lengths.dtype != torch.int32:
        raise ValueError("offsets must be int64 and lengths int32")
    N.check(N.load().stl_tx_hash_batch_device(
        ctypes.c_void_p(preimages.data_ptr()), ctypes.c_void_p(offsets.data_ptr()),
        ctypes.c_void_p(lengths.data_ptr()), n, ctypes.c_void_p(out_msg.data_ptr()), _stream_ptr(stream)),
        "stl_tx_hash_batch_device")
    return out_msg


def _check_rows(*ts):
    import torch
    for t in ts:
        if t is not None and (not t.is_cuda or not t.is_contiguous()):
            raise ValueError("device entry point needs contiguous CUDA tensors")
    if ts[1].dtype != torch.int64 or ts[2].dtype != torch.int32:
        raise ValueError("offsets must be int64 and lengths int32")


def tx_verify_batch_device(preimages, offsets, lengths, sig, pk, out_words=None, policy=POLICY_SODIUM_1_0_18,
                           stream=None):
    """stl_tx_verify_batch_device: the device-resident checkSign in one call --
    SHA512Half of each preimage and the verify, chunk by chunk over two
    streams -> int64 bitmap words (same bits as tx_hash_batch_device +
    verify_batch_device)."""
    import torch
    n = offsets.shape[0]
    if out_words is None:
        out_words = torch.empty(((n + 63) // 64,), dtype=torch.int64, device=preimages.device)
    _check_rows(preimages, offsets, lengths, sig, pk, out_words)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    N.check(N.load().stl_tx_verify_batch_device(p(preimages), p(offsets), p(lengths), p(sig), p(pk), n, p(out_words),
                                                policy, _stream_ptr(stream)), "stl_tx_verify_batch_device")
    return out_words


def signed_blob_verify_batch_device(blobs, offsets, lengths, out_words=None, tx_ids=False,
                                    policy=POLICY_SODIUM_1_0_18, stream=None, kind=None, out_status=None,
                                    out_ids=None):
    """stl_signed_blob_verify_batch_device: checkSign from serialized objects
    in HBM in one call -> dict of words (bitmap), status and (tx_ids or
    out_ids) tx_id."""
    import torch
    n = offsets.shape[0]
    dev = blobs.device
    if out_words is None:
        out_words = torch.empty(((n + 63) // 64,), dtype=torch.int64, device=dev)
    status = torch.empty((n,), dtype=torch.uint8, device=dev) if out_status is None else out_status
    tx_id = out_ids if out_ids is not None else (torch.empty((n, 32), dtype=torch.uint8, device=dev)
                                                 if tx_ids else None)
    # the kernels write raw bytes: a wider dtype would hold packed bytes the
    # caller misreads
    if status.dtype != torch.uint8 or (tx_id is not None and tx_id.dtype != torch.uint8):
        raise ValueError("out_status / out_ids must be torch.uint8")
    if tx_id is not None and tx_id.dim() > 1 and tx_id.shape[-1] != 32:
        raise ValueError("out_ids must be (n, 32) bytes")
    if status.numel() < n or (tx_id is not None and tx_id.numel() < 32 * n):
        raise ValueError("status / id buffers smaller than the batch")
    _check_rows(blobs, offsets, lengths, out_words, status, tx_id)
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    N.check(N.load().stl_signed_blob_verify_batch_device(
        N.STL_BLOB_TRANSACTION if kind is None else kind, p(blobs), p(offsets), p(lengths), n, p(out_words),
        p(status), p(tx_id), policy, _stream_ptr(stream)), "stl_signed_blob_verify_batch_device")
    return {"words": out_words, "status": status, "tx_id": tx_id}


def tx_blob_prepare_device(blobs, offsets, lengths, tx_ids=True, stream=None, kind=None):
    """Serialized transactions already in HBM (uint8 / int64 / int32 CUDA
    tensors) -> dict of msg (n,32), sig (n,64), pk (n,32), status (n,) and
    tx_id (n,32) tensors, asynchronously on ``stream``; follow with
    verify_batch_device(sig, msg, pk)."""
    import torch
    n = offsets.shape[0]
    dev = blobs.device
    out = {"msg": torch.empty((n, 32), dtype=torch.uint8, device=dev),
           "sig": torch.empty((n, 64), dtype=torch.uint8, device=dev),
           "pk": torch.empty((n, 32), dtype=torch.uint8, device=dev),
           "status": torch.empty((n,), dtype=torch.uint8, device=dev),
           "tx_id": torch.empty((n, 32), dtype=torch.uint8, device=dev) if tx_ids else None}
    for t in (blobs, offsets, lengths):
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("device entry point needs contiguous CUDA tensors")
    if offsets.dtype != torch.int64 or lengths.dtype != torch.int32:
        raise ValueError("offsets must be int64 and lengths int32")
    ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
    N.check(N.load().stl_signed_blob_prepare_device(
        N.STL_BLOB_TRANSACTION if kind is None else kind, ptr(blobs), ptr(offsets), ptr(lengths), n,
        ptr(out["msg"]), ptr(out["sig"]), ptr(out["pk"]), ptr(out["tx_id"]), ptr(out["status"]),
        _stream_ptr(stream)), "stl_signed_blob_prepare_device")
    return out


class Batcher:
    """stl_batcher (include/stl.h): single requests from any thread, run as
    device batches by max_batch / max_delay_us; ``submit`` / ``submit_tx``
    return a Future-like handle whose ``result()`` is the verdict
    (VERDICT_ACCEPT / VERDICT_REJECT / VERDICT_DEFER or a negative STL_E*)."""

    class Handle:
        def __init__(self):
            import threading
            self._ev = threading.Event()
            self.verdict = None

        def result(self, timeout=None):
            if not self._ev.wait(timeout):
                raise TimeoutError("verdict not delivered")
            return self.verdict

    def __init__(self, max_batch=4096, max_delay_us=1000, policy=POLICY_SODIUM_1_0_18):
        import threading
        self._lib = N.load()
        self._b = self._lib.stl_batcher_create(max_batch, max_delay_us, policy)
        if not self._b:
            raise ValueError("stl_batcher_create rejected its arguments")
        self._live = {}
        self._mu = threading.Lock()
        self._next = 0

        def done(ctx, verdict):
            with self._mu:
                h = self._live.pop(ctx)
            h.verdict = verdict
            h._ev.set()

        self._cb = N.VERDICT_FN(done)  # kept alive with the aggregator

    def _register(self):
        h = Batcher.Handle()
        with self._mu:
            self._next += 1
            key = self._next
            self._live[key] = h
        return key, h

    def submit(self, sig, msg32, pk):
        key, h = self._register()
        N.check(self._lib.stl_batcher_submit(self._b, bytes(sig), bytes(msg32), bytes(pk), self._cb, key),
                "stl_batcher_submit")
        return h

    def submit_tx(self, blob):
        key, h = self._register()
        blob = bytes(blob)
        N.check(self._lib.stl_batcher_submit_tx(self._b, blob, len(blob), self._cb, key), "stl_batcher_submit_tx")
        return h

    def flush(self):
        self._lib.stl_batcher_flush(self._b)

    def stats(self):
        v = [ctypes.c_uint64(0) for _ in range(3)]
        self._lib.stl_batcher_stats(self._b, *[ctypes.byref(x) for x in v])
        return {"submitted": v[0].value, "completed": v[1].value, "batches": v[2].value}

    def close(self):
        if self._b:
            self._lib.stl_batcher_destroy(self._b)
            self._b = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


VERDICT_REJECT, VERDICT_ACCEPT, VERDICT_DEFER = N.STL_VERDICT_REJECT, N.STL_VERDICT_ACCEPT, N.STL_VERDICT_DEFER


# ---- one process per GPU: the RCCL bitmap gather (include/stl.h) ----

def comm_unique_id():
    """stl_comm_unique_id: 128 bytes for rank 0 to hand to every rank."""
    buf = ctypes.create_string_buffer(128)
    N.check(N.load().stl_comm_unique_id(buf), "stl_comm_unique_id")
    return buf.raw


def comm_init_rank(nranks, rank, uid):
    uid = bytes(uid)
    if len(uid) != 128:
        raise ValueError("unique id is 128 bytes")
    N.check(N.load().stl_comm_init_rank(nranks, rank, uid), "stl_comm_init_rank")


def comm_destroy():
    N.load().stl_comm_destroy()


def comm_abort():
    """stl_comm_abort: tear the communicator down without waiting for peers."""
    N.load().stl_comm_abort()


def comm_sync(stream=None, timeout_ms=0):
    """stl_comm_sync: wait for ``stream`` under the RCCL deadline; raises
    StlError (STL_ERCCL) after aborting the communicator if a gather stalls."""
    N.check(N.load().stl_comm_sync(_stream_ptr(stream), int(timeout_ms)), "stl_comm_sync")


def comm_info():
    """stl_comm_info: (nranks, rank) as RCCL reports them (ncclCommCount /
    ncclCommUserRank) for the communicator libstl gathers over."""
    nr, r = ctypes.c_int(0), ctypes.c_int(0)
    N.check(N.load().stl_comm_info(ctypes.byref(nr), ctypes.byref(r)), "stl_comm_info")
    return nr.value, r.value


def bitmap_gather_device(words, out_words=None, root=0, stream=None):
    """stl_bitmap_gather_device: every rank's int64 bitmap words (CUDA tensor of
    words_per_rank words) into out_words (nranks*words_per_rank) on rank
    ``root`` (root < 0: all ranks)."""
    ptr = ctypes.c_void_p(out_words.data_ptr()) if out_words is not None else None
    N.check(N.load().stl_bitmap_gather_device(ctypes.c_void_p(words.data_ptr()), words.numel(), ptr, root,
                                              _stream_ptr(stream)), "stl_bitmap_gather_device")
    return out_words


def bitmap_gatherv_device(words, word_offsets, out_words=None, root=0, stream=None):
    """stl_bitmap_gatherv_device: rank r's int64 words (word_offsets[r+1] -
    word_offsets[r] of them) into out_words[word_offsets[r]:] on rank
    ``root``; word_offsets has nranks+1 entries, the same on every rank."""
    offs = np.ascontiguousarray(word_offsets, dtype=np.uint64)
    ptr = ctypes.c_void_p(out_words.data_ptr()) if out_words is not None else None
    wptr = ctypes.c_void_p(words.data_ptr()) if words.numel() else None
    N.check(N.load().stl_bitmap_gatherv_device(wptr, words.numel(), ptr, _buf(offs), root, _stream_ptr(stream)),
            "stl_bitmap_gatherv_device")
    return out_words


# ---- statistics (include/stl.h stl_get_stats) ----

class Stats(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("batches", ctypes.c_uint64), ("signatures", ctypes.c_uint64), ("errors", ctypes.c_uint64),
                ("host_ns", ctypes.c_uint64), ("gather_ns", ctypes.c_uint64),
                ("accepted", ctypes.c_uint64), ("full_length_lanes", ctypes.c_uint64),
                ("phase_ns", ctypes.c_uint64 * 4), ("phase_chunks", ctypes.c_uint64),
                ("auto_dedup_chunks", ctypes.c_uint64)]


# stl_stats.phase_ns: [0] the first phase-1 kernel -- all of phase 1 when it
# runs as one kernel (the default), the SHA-512 + lattice kernel when split;
# [1] the point-decoding kernel when split, the key-dedup kernels; [2] the main
# kernel; [3] the full-length fallback kernel
PHASES = ("phase1", "point", "main", "fallback")


def get_stats():
    """Counters of include/stl.h stl_get_stats; ``phase_ns`` is a dict of the
    summed kernel time per verify phase (zero unless phase timing is on)."""
    st = Stats()
    st.struct_size = ctypes.sizeof(Stats)
    N.check(N.load().stl_get_stats(ctypes.byref(st)), "stl_get_stats")
    out = {name: getattr(st, name) for name, _ in Stats._fields_
           if name not in ("struct_size", "reserved", "phase_ns")}
    out["phase_ns"] = dict(zip(PHASES, list(st.phase_ns)))
    return out


def reset_stats():
    N.load().stl_reset_stats()


def set_phase_timing(on):
    """Per-phase HIP-event timing of the verify launches (stl_set_phase_timing);
    returns the previous setting."""
    return bool(N.load().stl_set_phase_timing(1 if on else 0))


# ---- testing hooks ----

def debug_fault_after(calls):
    """stl_debug_fault_after: the HIP/RCCL call after ``calls`` more fails (one shot)."""
    N.load().stl_debug_fault_after(calls)


def debug_verify_k_device(sig, k, pk, out_words=None, policy=POLICY_SODIUM_1_0_18, stream=None):
    """stl_debug_verify_k_device: verify with given k (n,32) instead of hashing."""
    import torch
    n = sig.shape[0]
    if out_words is None:
        out_words = torch.empty((n + 63) // 64, dtype=torch.int64, device=sig.device)
    N.check(N.load().stl_debug_verify_k_device(
        ctypes.c_void_p(sig.data_ptr()), ctypes.c_void_p(k.data_ptr()), ctypes.c_void_p(pk.data_ptr()), n,
        ctypes.c_void_p(out_words.data_ptr()), policy, _stream_ptr(stream)), "stl_debug_verify_k_device")
    return out_words


TUNE_FUSED_PREP, TUNE_MAIN_QUEUE = N.STL_TUNE_FUSED_PREP, N.STL_TUNE_MAIN_QUEUE
TUNE_STREAMS, TUNE_CHUNK_LOG2 = N.STL_TUNE_STREAMS, N.STL_TUNE_CHUNK_LOG2
TUNE_BYTE_SHARDS = N.STL_TUNE_BYTE_SHARDS
TUNE_QUAD = N.STL_TUNE_QUAD
TUNE_STREAM_WORKSPACES = N.STL_TUNE_STREAM_WORKSPACES
TUNE_RCCL_TIMEOUT_MS = N.STL_TUNE_RCCL_TIMEOUT_MS
TUNE_LONG_HASH = N.STL_TUNE_LONG_HASH
TUNE_SHARED_KEYS = N.STL_TUNE_SHARED_KEYS
TUNE_WIDE_MIN_ROWS = N.STL_TUNE_WIDE_MIN_ROWS
TUNE_R_AHEAD = N.STL_TUNE_R_AHEAD
TUNE_FIRST_CHUNK = N.STL_TUNE_FIRST_CHUNK


def debug_tuning(key, value):
    """stl_debug_tuning: process-wide execution setting (same accept bits
    whatever the value); returns the previous value."""
    rc = N.load().stl_debug_tuning(key, value)
    if rc < 0:
        raise N.StlError(rc, "stl_debug_tuning")
    return rc


def release_stream(stream):
    """stl_release_stream: free libstl's context of a caller stream (a torch
    stream) on the current device."""
    N.check(N.load().stl_release_stream(_stream_ptr(stream)), "stl_release_stream")


def stream_contexts():
    """Caller-stream contexts libstl keeps on the current device
    (at most debug_tuning(TUNE_STREAM_WORKSPACES, -1))."""
    rc = N.load().stl_debug_stream_contexts()
    if rc < 0:
        N.check(rc, "stl_debug_stream_contexts")
    return rc


def clock_stamp(nwg=256, stream=None):
    """stl_debug_clock_stamp: (nwg, 4) int64 CUDA tensor of {shader cycle
    counter, 100 MHz counter, XCC_ID, HW_ID} per one-wave workgroup, enqueued
    on ``stream`` (bench.py's clock_ghz)."""
    import torch
    out = torch.zeros((nwg, 4), dtype=torch.int64, device="cuda")
    N.check(N.load().stl_debug_clock_stamp(ctypes.c_void_p(out.data_ptr()), nwg, _stream_ptr(stream)),
            "stl_debug_clock_stamp")
    return out


def clock_ghz(start, end):
    """Average shader clock (GHz) between two clock_stamp results (numpy or
    torch (nwg, 4)).  Each CU keeps its own cycle counter (tools/clock_probe.py:
    counters of one XCD differ by ~1e8 cycles at one instant), so stamps are
    matched per CU -- XCC_ID and HW_ID bits 8-15 (CU, SH, SE) -- and the clock
    of each CU is its cycle delta over its 100 MHz delta.  Returns (median over
    the CUs found in both stamps, {xcc: median over its CUs}, CUs matched)."""
    a = start.cpu().numpy() if hasattr(start, "cpu") else np.asarray(start)
    b = end.cpu().numpy() if hasattr(end, "cpu") else np.asarray(end)

    def by_cu(x):
        d = {}
        for t, rt, xcc, hw in x.tolist():
            d.setdefault((int(xcc) & 0xF, (int(hw) >> 8) & 0xFF), []).append((t, rt))
        return {k: (float(np.median([v[0] for v in vs])), float(np.median([v[1] for v in vs])))
                for k, vs in d.items()}
    sa, sb = by_cu(a), by_cu(b)
    per_cu = {}
    for k in sorted(set(sa) & set(sb)):
        dr = sb[k][1] - sa[k][1]
        if dr > 0:
            per_cu[k] = (sb[k][0] - sa[k][0]) / dr * 0.1
    if not per_cu:
        return None, {}, 0
    per_xcc = {}
    for (xcc, _), v in per_cu.items():
        per_xcc.setdefault(xcc, []).append(v)
    vals = sorted(per_cu.values())
    return vals[len(vals) // 2], {x: float(np.median(v)) for x, v in sorted(per_xcc.items())}, len(per_cu)


def execution_settings():
    """The current stl_debug_tuning values."""
    lib = N.load()
    return {name: lib.stl_debug_tuning(key, -1) for name, key in (
        ("fused_prep", TUNE_FUSED_PREP), ("main_queue", TUNE_MAIN_QUEUE), ("streams", TUNE_STREAMS),
        ("chunk_log2", TUNE_CHUNK_LOG2), ("quad", TUNE_QUAD), ("long_hash", TUNE_LONG_HASH),
        ("shared_keys", TUNE_SHARED_KEYS), ("wide_min_rows", TUNE_WIDE_MIN_ROWS),
        ("r_ahead", TUNE_R_AHEAD), ("first_chunk", TUNE_FIRST_CHUNK))}


def sign_batch_device(seed, msg, stream=None):
    """RFC 8032 keypair(seed) + detached signature over msg, on the GPU.
    seed (n,32), msg (n,32) uint8 CUDA tensors -> (pk (n,32), sig (n,64))."""
    import torch
    n = seed.shape[0]
    pk = torch.empty((n, 32), dtype=torch.uint8, device=seed.device)
    sig = torch.empty((n, 64), dtype=torch.uint8, device=seed.device)
    N.check(N.load().stl_ed25519_sign_batch_device(
        ctypes.c_void_p(seed.data_ptr()), ctypes.c_void_p(msg.data_ptr()), n, ctypes.c_void_p(pk.data_ptr()),
        ctypes.c_void_p(sig.data_ptr()), _stream_ptr(stream)), "stl_ed25519_sign_batch_device")
    return pk, sig


def sign_adversarial_device(seed, msg, cls, param, stream=None):
    """Test data: sign_batch_device, then rows with cls (n,) uint8 in 1..11
    mutated into SURVEY Appendix-B class B<cls> with parameter param (n,)
    int32 (tests/datasets.py).  -> (pk, sig, msg) CUDA tensors."""
    import torch
    n = seed.shape[0]
    pk = torch.empty((n, 32), dtype=torch.uint8, device=seed.device)
    sig = torch.empty((n, 64), dtype=torch.uint8, device=seed.device)
    mo = torch.empty((n, 32), dtype=torch.uint8, device=seed.device)
    for t in (seed, msg, cls, param):
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("device entry point needs contiguous CUDA tensors")
    N.check(N.load().stl_debug_sign_adversarial_device(
        ctypes.c_void_p(seed.data_ptr()), ctypes.c_void_p(msg.data_ptr()), ctypes.c_void_p(cls.data_ptr()),
        ctypes.c_void_p(param.data_ptr()), n, ctypes.c_void_p(pk.data_ptr()), ctypes.c_void_p(sig.data_ptr()),
        ctypes.c_void_p(mo.data_ptr()), _stream_ptr(stream)), "stl_debug_sign_adversarial_device")
    return pk, sig, mo


def words_to_bool(words, n):
    """int64 bitmap words (torch or numpy) -> bool[n] numpy."""
    arr = words.cpu().numpy() if hasattr(words, "cpu") else np.asarray(words)
    return np.unpackbits(arr.astype("<i8").view(np.uint8), bitorder="little")[:n].astype(bool)
