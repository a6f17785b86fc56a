"""ctypes binding of libstl.so (the C ABI in include/stl.h).

The shared library is built in-tree by ``stellard_amd.build`` (hipcc,
--offload-arch=gfx950).  There is no Python or CPU fallback: if the library is
missing this module raises, so a GPU run can never silently verify on the host.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("STL_LIB_PATH") or os.path.join(_HERE, "libstl.so")

STL_OK = 0
STL_EINVAL = -22
STL_ENODEV = -19
STL_ENOMEM = -12
STL_EHIP = -1000
STL_ERCCL = -1001

# stl_config.flags
STL_CFG_RCCL_GATHER = 0x1
STL_CFG_NO_RCCL = 0x2

# signed-object kinds of the blob entry points
STL_BLOB_TRANSACTION = 0
STL_BLOB_VALIDATION = 1

STL_POLICY_SODIUM_1_0_18 = 0x0
STL_POLICY_STELLARD_1_0_0 = 0x1
STL_POLICY_MASK = 0x1
STL_REQUIRE_S_LT_L = 0x2
STL_FULL_LENGTH = 0x4
STL_DEDUP_KEYS = 0x8
STL_ONE_LANE = 0x10
STL_NO_AUTO_DEDUP = 0x20
STL_DEBUG_RAW_PREDICATE = 0x80000000  # test-only: no S < L (stl.h)

# stl_debug_tuning keys
STL_TUNE_FUSED_PREP = 0
STL_TUNE_MAIN_QUEUE = 1
STL_TUNE_STREAMS = 2
STL_TUNE_CHUNK_LOG2 = 3
STL_TUNE_BYTE_SHARDS = 4
STL_TUNE_QUAD = 5
STL_TUNE_STREAM_WORKSPACES = 6
STL_TUNE_RCCL_TIMEOUT_MS = 7
STL_TUNE_LONG_HASH = 8
STL_TUNE_SHARED_KEYS = 9
STL_TUNE_WIDE_MIN_ROWS = 10
STL_TUNE_R_AHEAD = 11
STL_TUNE_FIRST_CHUNK = 12

# per-transaction status of the serialized-transaction entry points
STL_TX_OK = 0
STL_TX_DEFERRED = 1
STL_TX_MALFORMED = 2

# Every entry point include/stl.h declares: (name, restype, argtypes)
_P = ctypes.c_void_p
_U8P = ctypes.c_void_p
SYMBOLS = [
    ("stl_init", ctypes.c_int, [_P]),
    ("stl_shutdown", None, []),
    ("stl_device_count", ctypes.c_int, []),
    ("stl_version", ctypes.c_char_p, []),
    ("stl_strerror", ctypes.c_char_p, [ctypes.c_int]),
    ("stl_ed25519_verify_detached", ctypes.c_int, [_U8P, _U8P, ctypes.c_ulonglong, _U8P]),
    ("stl_ed25519_verify_batch", ctypes.c_int, [_U8P, _U8P, _U8P, ctypes.c_size_t, _U8P, ctypes.c_uint32]),
    ("stl_tx_verify_batch", ctypes.c_int,
     [_U8P, _P, _P, _U8P, _U8P, ctypes.c_size_t, _U8P, ctypes.c_uint32]),
    ("stl_ed25519_verify_batch_device", ctypes.c_int,
     [_U8P, _U8P, _U8P, ctypes.c_size_t, _P, ctypes.c_uint32, _P]),
    ("stl_tx_hash_batch_device", ctypes.c_int, [_U8P, _P, _P, ctypes.c_size_t, _U8P, _P]),
    ("stl_ed25519_sign_batch_device", ctypes.c_int, [_U8P, _U8P, ctypes.c_size_t, _U8P, _U8P, _P]),
    ("stl_tx_blob_verify_batch", ctypes.c_int,
     [_U8P, _P, _P, ctypes.c_size_t, _U8P, _U8P, _U8P, ctypes.c_uint32]),
    ("stl_tx_blob_prepare_device", ctypes.c_int,
     [_U8P, _P, _P, ctypes.c_size_t, _U8P, _U8P, _U8P, _U8P, _U8P, _P]),
    ("stl_tx_verify_batch_device", ctypes.c_int,
     [_U8P, _P, _P, _U8P, _U8P, ctypes.c_size_t, _P, ctypes.c_uint32, _P]),
    ("stl_signed_blob_verify_batch_device", ctypes.c_int,
     [ctypes.c_uint32, _U8P, _P, _P, ctypes.c_size_t, _P, _U8P, _U8P, ctypes.c_uint32, _P]),
    ("stl_batcher_create", ctypes.c_void_p, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]),
    ("stl_batcher_submit", ctypes.c_int, [_P, _U8P, _U8P, _U8P, _P, _P]),
    ("stl_batcher_submit_tx", ctypes.c_int, [_P, _U8P, ctypes.c_size_t, _P, _P]),
    ("stl_batcher_flush", None, [_P]),
    ("stl_batcher_stats", None, [_P, _P, _P, _P]),
    ("stl_batcher_destroy", None, [_P]),
    ("stl_signed_blob_verify_batch", ctypes.c_int,
     [ctypes.c_uint32, _U8P, _P, _P, ctypes.c_size_t, _U8P, _U8P, _U8P, ctypes.c_uint32]),
    ("stl_signed_blob_prepare_device", ctypes.c_int,
     [ctypes.c_uint32, _U8P, _P, _P, ctypes.c_size_t, _U8P, _U8P, _U8P, _U8P, _U8P, _P]),
    ("stl_comm_unique_id", ctypes.c_int, [_U8P]),
    ("stl_comm_init_rank", ctypes.c_int, [ctypes.c_int, ctypes.c_int, _U8P]),
    ("stl_comm_destroy", None, []),
    ("stl_comm_abort", None, []),
    ("stl_comm_sync", ctypes.c_int, [_P, ctypes.c_int]),
    ("stl_comm_info", ctypes.c_int, [_P, _P]),
    ("stl_bitmap_gather_device", ctypes.c_int, [_P, ctypes.c_size_t, _P, ctypes.c_int, _P]),
    ("stl_bitmap_gatherv_device", ctypes.c_int, [_P, ctypes.c_size_t, _P, _P, ctypes.c_int, _P]),
    ("stl_shard_range", None, [ctypes.c_size_t, ctypes.c_int, ctypes.c_int, _P, _P]),
    ("stl_shard_range_bytes", None, [_P, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, _P, _P]),
    ("stl_debug_fault_after", None, [ctypes.c_longlong]),
    ("stl_get_stats", ctypes.c_int, [_P]),
    ("stl_reset_stats", None, []),
    ("stl_set_phase_timing", ctypes.c_int, [ctypes.c_int]),
    ("stl_debug_verify_k_device", ctypes.c_int, [_U8P, _U8P, _U8P, ctypes.c_size_t, _P, ctypes.c_uint32, _P]),
    ("stl_debug_tuning", ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
    ("stl_debug_stream_contexts", ctypes.c_int, []),
    ("stl_debug_clock_stamp", ctypes.c_int, [_P, ctypes.c_uint32, _P]),
    ("stl_release_stream", ctypes.c_int, [_P]),
    ("stl_debug_sign_adversarial_device", ctypes.c_int,
     [_U8P, _U8P, _U8P, _P, ctypes.c_size_t, _U8P, _U8P, _U8P, _P]),
]

VERDICT_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int)
STL_VERDICT_REJECT, STL_VERDICT_ACCEPT, STL_VERDICT_DEFER = 0, 1, 2


class StlError(RuntimeError):
    def __init__(self, rc, what=""):
        self.rc = rc
        super().__init__(f"libstl error {rc} ({strerror(rc)}) {what}".strip())


_lib = None


def load():
    """Load libstl.so and bind every exported symbol; raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(libstl has no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SYMBOLS:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def strerror(rc):
    try:
        return load().stl_strerror(rc).decode()
    except Exception:  # noqa: BLE001 - used while formatting an error
        return "?"


def check(rc, what=""):
    if rc != STL_OK:
        raise StlError(rc, what)
    return rc
