"""The C-ABI library loads and exports every symbol include/stl.h declares
(no compute calls: this runs without a GPU)."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    with open(os.path.join(ROOT, "include", "stl.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(stl_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ("stl_init", "stl_ed25519_verify_detached", "stl_ed25519_verify_batch", "stl_tx_verify_batch",
              "stl_ed25519_verify_batch_device"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from stellard_amd import _native
    lib = _native.load()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing
    bound = {name for name, _, _ in _native.SYMBOLS}
    assert set(declared_symbols()) == bound


def test_python_constants_match_header():
    """Every numeric STL_* macro of include/stl.h has the same value in
    stellard_amd/_native.py (the ctypes mirror the tests and bench use)."""
    from stellard_amd import _native
    with open(os.path.join(ROOT, "include", "stl.h")) as f:
        text = f.read()
    macros = dict(re.findall(r"#define\s+(STL_[A-Z0-9_]+)\s+\(?(-?(?:0x[0-9a-fA-F]+|\d+))u?\)?", text))
    assert len(macros) > 20
    missing = sorted(m for m in macros if m != "STL_ABI_VERSION" and not hasattr(_native, m))
    assert not missing, missing
    for m, v in macros.items():
        if hasattr(_native, m):
            assert getattr(_native, m) == int(v, 0), m


def test_library_is_gfx950_code_object():
    from stellard_amd import _native
    with open(_native.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob


def test_no_cpu_verify_without_gpu():
    """Without a GPU the library reports ENODEV -- it never verifies on the host."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from stellard_amd import _native
    lib = _native.load()
    rc = lib.stl_ed25519_verify_detached(bytes(64), bytes(32), 32, bytes(32))
    assert rc == _native.STL_ENODEV


def test_batcher_without_device_completes_every_request_with_an_error():
    """The aggregator (f2) on a GPU-less box: every request completes exactly
    once, with a negative error (the caller's fallback signal), never a
    reject; batches respect max_batch; flush waits for all; threads may submit
    concurrently."""
    import threading

    from stellard_amd import verify as V
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by the gpu tests")
    with V.Batcher(max_batch=16, max_delay_us=200) as b:
        handles = []
        lock = threading.Lock()

        def worker(k):
            for i in range(40):
                h = b.submit(bytes([k]) * 64, bytes([i]) * 32, bytes(32)) if i % 3 else b.submit_tx(bytes(200))
                with lock:
                    handles.append(h)

        ts = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        b.flush()
        st = b.stats()
        assert st["submitted"] == 160 and st["completed"] == 160
        assert st["batches"] >= 160 // 16
        for h in handles:
            assert h.result(timeout=5) < 0


def test_batcher_rejects_bad_arguments():
    from stellard_amd import _native as N
    lib = N.load()
    assert not lib.stl_batcher_create(0, 100, 0)
    assert not lib.stl_batcher_create(16, 100, 0x80)
    assert lib.stl_batcher_submit(None, bytes(64), bytes(32), bytes(32), None, None) == N.STL_EINVAL


def test_flag_validation():
    """Every STL_* verify flag of stl.h is accepted (STL_ONE_LANE included);
    an unknown bit is STL_EINVAL before any device work, on every box."""
    import ctypes
    from stellard_amd import _native as N
    lib = N.load()
    sig, msg, pk, bm = bytes(64), bytes(32), bytes(32), ctypes.create_string_buffer(1)
    for flags in (0, N.STL_POLICY_STELLARD_1_0_0, N.STL_FULL_LENGTH, N.STL_DEDUP_KEYS, N.STL_ONE_LANE,
                  N.STL_DEDUP_KEYS | N.STL_ONE_LANE, N.STL_NO_AUTO_DEDUP):
        assert lib.stl_ed25519_verify_batch(sig, msg, pk, 1, bm, flags) != N.STL_EINVAL, flags
    assert lib.stl_ed25519_verify_batch(sig, msg, pk, 1, bm, 0x40) == N.STL_EINVAL
    b = lib.stl_batcher_create(16, 100, N.STL_ONE_LANE)
    assert b
    lib.stl_batcher_destroy(b)


def test_blob_call_rejects_wide_status_and_id_buffers():
    """the blob call's kernels write raw bytes into out_status and
    out_ids, so a wider dtype (or ids not 32 bytes wide) is refused before any
    device call -- a caller would otherwise read packed bytes as elements."""
    torch = pytest.importorskip("torch")
    from stellard_amd import verify as V
    n = 4
    blobs = torch.zeros(64, dtype=torch.uint8)
    off = torch.zeros(n, dtype=torch.int64)
    ln = torch.zeros(n, dtype=torch.int32)
    with pytest.raises(ValueError, match="uint8"):
        V.signed_blob_verify_batch_device(blobs, off, ln, out_status=torch.zeros(n, dtype=torch.int32))
    with pytest.raises(ValueError, match="uint8"):
        V.signed_blob_verify_batch_device(blobs, off, ln, out_status=torch.zeros(n, dtype=torch.uint8),
                                          out_ids=torch.zeros((n, 4), dtype=torch.int64))
    with pytest.raises(ValueError, match=r"\(n, 32\)"):
        V.signed_blob_verify_batch_device(blobs, off, ln, out_status=torch.zeros(n, dtype=torch.uint8),
                                          out_ids=torch.zeros((n, 64), dtype=torch.uint8))
