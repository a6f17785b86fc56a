"""GPU tests of libstl's execution settings (stl_debug_tuning): the fused
phase-1 kernel, the main kernel's unit queue, and chunks over concurrent
streams -- every setting must give the same accept bits as the two-kernel,
grid-stride, one-stream path of round 2, and those bits are the oracle's.

Run on an MI355X:  python -u -m pytest tests -m gpu -x -v --timeout 120
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def stl(torch_cuda):
    from stellard_amd import verify
    verify.init()
    return verify


SETTINGS = [  # (fused_prep, main_queue, streams, chunk_log2[, first chunk rows])
    (0, 0, 1, 18), (1, 0, 1, 18), (0, 1, 1, 18), (1, 1, 1, 18),
    (1, 1, 2, 18), (1, 1, 4, 18), (1, 1, 3, 17), (1, 1, 4, 16), (0, 0, 2, 19), (1, 1, 2, 20), (1, 1, 2, 0),
    (1, 1, 2, 15), (1, 1, 3, 15),  # lane-pair chunks on concurrent streams
    (1, 1, 2, 0, 65536), (1, 1, 2, 0, 32768), (1, 1, 3, 17, 100032),  # a smaller first chunk (STL_TUNE_FIRST_CHUNK)
]


def _apply(stl, v):
    old = []
    v = tuple(v) + (0,) * (5 - len(v))
    for key, val in zip((stl.TUNE_FUSED_PREP, stl.TUNE_MAIN_QUEUE, stl.TUNE_STREAMS, stl.TUNE_CHUNK_LOG2,
                         stl.TUNE_FIRST_CHUNK), v):
        old.append(stl.debug_tuning(key, val))
    return tuple(old)


@pytest.fixture(scope="module")
def batch(stl, torch_cuda, golden):
    """600,037 rows: GPU-signed valid signatures, 1 % with a flipped message
    byte, and every 97th row a golden vector (all Appendix-B classes)."""
    torch = torch_cuda
    n = 600_037
    rng = np.random.default_rng(77)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pk, sig = stl.sign_batch_device(torch.from_numpy(seeds).cuda(), torch.from_numpy(msgs).cuda())
    sig, pk = sig.cpu().numpy(), pk.cpu().numpy()
    flip = rng.choice(n, n // 100, replace=False)
    msgs[flip, 3] ^= 0x10
    rows = np.arange(0, n, 97)
    pick = rng.integers(0, golden["sig"].shape[0], rows.size)
    sig[rows], msgs[rows], pk[rows] = golden["sig"][pick], golden["msg"][pick], golden["pk"][pick]
    exp_golden = golden["expected_sodium_1_0_18"][pick].astype(bool)
    d = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (sig, msgs, pk)]
    return n, d, (sig, msgs, pk), rows, exp_golden, flip


def _run(stl, torch, d, n, policy=0):
    w = stl.verify_batch_device(*d, policy=policy)
    torch.cuda.synchronize()
    return stl.words_to_bool(w, n)


def test_settings_same_bits(stl, torch_cuda, batch, oracle):
    torch = torch_cuda
    n, d, host, rows, exp_golden, flip = batch
    old = _apply(stl, SETTINGS[0])
    try:
        ref = _run(stl, torch, d, n)
        # the reference path's bits are the oracle's: golden rows exactly, the
        # flipped rows rejected, and a 20,000-row sample re-checked
        assert np.array_equal(ref[rows], exp_golden)
        assert not ref[np.setdiff1d(flip, rows)].any()
        sample = np.random.default_rng(5).choice(n, 20_000, replace=False)
        assert np.array_equal(ref[sample], oracle.verify_batch(*(a[sample] for a in host)))
        for v in SETTINGS[1:]:
            _apply(stl, v)
            got = _run(stl, torch, d, n)
            assert np.array_equal(got, ref), (v, np.nonzero(got != ref)[0][:8])
    finally:
        _apply(stl, old)


@pytest.mark.parametrize("flags", ["full_length", "dedup", "policy100"])
def test_settings_same_bits_with_flags(stl, torch_cuda, batch, flags):
    """The flag paths under concurrent streams: full-length lanes, key dedup
    (each stream's workspace has its own key tables) and the 1.0.0 policy."""
    torch = torch_cuda
    n, d, host, rows, exp_golden, flip = batch
    pol = {"full_length": stl.FULL_LENGTH, "dedup": stl.DEDUP_KEYS, "policy100": stl.POLICY_STELLARD_1_0_0}[flags]
    old = _apply(stl, SETTINGS[0])
    try:
        ref = _run(stl, torch, d, n, pol)
        for v in ((1, 1, 1, 18), (1, 1, 4, 16), (1, 1, 2, 18), (0, 1, 2, 17), (1, 1, 2, 0, 65536)):
            _apply(stl, v)
            assert np.array_equal(_run(stl, torch, d, n, pol), ref), (flags, v)
    finally:
        _apply(stl, old)
    if flags != "policy100":
        assert np.array_equal(ref, _run(stl, torch, d, n))


def test_streams_with_caller_stream_and_phase_timing(stl, torch_cuda, batch):
    """A call on a side stream forks the library's streams from it and joins
    them back: work queued after the call on the same stream sees the whole
    bitmap.  Under the phase clock the chunks run on one stream and every
    chunk is timed."""
    torch = torch_cuda
    n, d, host, rows, exp_golden, flip = batch
    old = _apply(stl, (1, 1, 4, 16))
    try:
        ref = _run(stl, torch, d, n)
        s = torch.cuda.Stream()
        w = torch.zeros((n + 63) // 64, dtype=torch.int64, device="cuda")
        with torch.cuda.stream(s):
            for _ in range(3):
                w.zero_()
                stl.verify_batch_device(*d, out_words=w, stream=s)
            total = w.clone()  # on s: after the joined streams
        torch.cuda.synchronize()
        assert np.array_equal(stl.words_to_bool(total, n), ref)
        stl.reset_stats()
        stl.set_phase_timing(True)
        try:
            assert np.array_equal(_run(stl, torch, d, n), ref)
            st = stl.get_stats()
        finally:
            stl.set_phase_timing(False)
        assert st["phase_chunks"] == 1  # n < 2^20: one chunk, kernels one after another
        assert st["phase_ns"]["main"] > 0
    finally:
        _apply(stl, old)


def test_host_api_streams_same_bits(stl, torch_cuda, batch):
    """The host batch API runs its 64K-signature chunks on one kernel stream,
    or (streams > 1, the default) the odd chunks on a second stream with their
    own verify workspace: same bits as the device API either way, with and
    without key dedup (per-stream key tables)."""
    torch = torch_cuda
    n, d, host, rows, exp_golden, flip = batch
    old = _apply(stl, SETTINGS[0])
    try:
        ref = _run(stl, torch, d, n)
        ref_dedup = _run(stl, torch, d, n, stl.DEDUP_KEYS)
        for streams in (1, 2):
            stl.debug_tuning(stl.TUNE_STREAMS, streams)
            assert np.array_equal(stl.verify_batch(*host), ref), streams
            assert np.array_equal(stl.verify_batch(*host, policy=stl.DEDUP_KEYS), ref_dedup), streams
    finally:
        _apply(stl, old)


def test_host_tx_api_streams_same_bits(stl, torch_cuda):
    """stl_tx_verify_batch over 300,001 preimages (five 64K chunks: the
    odd ones on the second stream with its own hash work counter): signatures
    made on the GPU over SHA512Half of each preimage (hashlib), a 1 % sample
    of rows signed over a different hash; same bits with one and two streams,
    equal to the expectation."""
    import hashlib
    torch = torch_cuda
    n = 300_001
    rng = np.random.default_rng(31)
    lens = rng.integers(100, 400, n)
    blob = rng.integers(0, 256, int(lens.sum()), dtype=np.uint8).tobytes()
    offs = np.concatenate(([0], np.cumsum(lens)[:-1]))
    pres = [b"STX\0" + blob[o:o + ln] for o, ln in zip(offs, lens)]
    h = np.frombuffer(b"".join(hashlib.sha512(p).digest()[:32] for p in pres), np.uint8).reshape(n, 32).copy()
    bad = rng.choice(n, n // 100, replace=False)
    h[bad, 0] ^= 1
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pk, sig = stl.sign_batch_device(torch.from_numpy(seeds).cuda(), torch.from_numpy(h).cuda())
    sig, pk = sig.cpu().numpy(), pk.cpu().numpy()
    exp = np.ones(n, bool)
    exp[bad] = False
    old = stl.debug_tuning(stl.TUNE_STREAMS, 1)
    try:
        for streams in (1, 2):
            stl.debug_tuning(stl.TUNE_STREAMS, streams)
            got = stl.tx_verify_batch(pres, sig, pk)
            assert np.array_equal(got, exp), (streams, np.nonzero(got != exp)[0][:8])
    finally:
        stl.debug_tuning(stl.TUNE_STREAMS, old)


def test_tuning_rejects_bad_values(stl):
    from stellard_amd import _native as N
    lib = N.load()
    for key, bad in ((stl.TUNE_FUSED_PREP, 2), (stl.TUNE_FUSED_PREP, 3), (stl.TUNE_FUSED_PREP, -2), (stl.TUNE_MAIN_QUEUE, -2), (stl.TUNE_STREAMS, 0),
                     (stl.TUNE_STREAMS, 5), (stl.TUNE_CHUNK_LOG2, 14), (stl.TUNE_CHUNK_LOG2, 21), (stl.TUNE_QUAD, 4), (stl.TUNE_QUAD, -2), (99, 1)):
        assert lib.stl_debug_tuning(key, bad) == N.STL_EINVAL, (key, bad)
    assert stl.execution_settings()["streams"] in (1, 2, 3, 4)


@pytest.mark.timeout(300)
def test_overlap_survives_caller_streams(stl, torch_cuda):
    """libstl's streams come from a fixed per-device pool made in
    stl_init, so streams a caller creates afterwards (here: a host API call,
    then two caller streams with work on them) cannot take the hardware queue
    of the stream a device-resident call spreads its chunks onto.  A 1M launch
    on the caller's stream must stay at least 2 % below the serial sum of its
    kernels (phase clock: prep + main + fallback one after another)."""
    torch = torch_cuda
    n = 1 << 20
    rng = np.random.default_rng(404)
    seeds = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
    msgs = torch.from_numpy(rng.integers(0, 256, (n, 32), dtype=np.uint8)).cuda()
    pk, sig = stl.sign_batch_device(seeds, msgs)
    h = [a[:70_000].cpu().numpy() for a in (sig, msgs, pk)]
    assert stl.verify_batch(*h).all()  # the host API first
    extra = [torch.cuda.Stream() for _ in range(2)]
    for s in extra:
        with torch.cuda.stream(s):
            torch.ones(1 << 20, device="cuda").sum()
    torch.cuda.synchronize()
    old = _apply(stl, (1, 1, 2, 18))  # the default execution
    words = torch.empty(n // 64, dtype=torch.int64, device="cuda")
    try:
        def launches(k):
            stream = torch.cuda.current_stream()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(k + 1)]
            ev[0].record(stream)
            for i in range(k):
                stl.verify_batch_device(sig, msgs, pk, out_words=words, stream=stream)
                ev[i + 1].record(stream)
            torch.cuda.synchronize()
            return [ev[i].elapsed_time(ev[i + 1]) for i in range(k)]

        launches(3)
        overlapped = float(np.median(launches(10)))
        assert stl.words_to_bool(words, n).all()
        stl.reset_stats()
        stl.set_phase_timing(True)
        try:
            launches(10)
            st = stl.get_stats()
        finally:
            stl.set_phase_timing(False)
        serial = sum(st["phase_ns"].values()) / max(1, st["phase_chunks"]) / 1e6
        print(f"launch {overlapped:.3f} ms, serial kernel sum {serial:.3f} ms")
        assert overlapped <= 0.98 * serial, (overlapped, serial)
    finally:
        _apply(stl, old)

