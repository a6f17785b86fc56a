"""SHA512Half of transaction signing preimages (Serializer.cpp:354-360 via
STObject::getSigningHash, SerializedObject.cpp:444-450) with the
word-granular reader the tx-hash kernel uses (stl_sha512.h ByteStream:
aligned dword loads shifted by v_alignbyte, FIPS 180-4 padding applied in
registers), compiled for the host by tests/native/hostemu.cpp and checked
against hashlib on every length 0..600 at every byte alignment and on
config-5 lengths (100 B - 4 KB)."""
import ctypes
import hashlib

import numpy as np
import pytest

from tests import oracle_bind


@pytest.fixture(scope="module")
def emu():
    return oracle_bind.load_hostemu()


def _half(emu, buf, off, n):
    out = ctypes.create_string_buffer(32)
    emu.hostemu_sha512_half(ctypes.c_void_p(buf.ctypes.data + off), n, out)
    return out.raw


def test_every_length_and_alignment(emu):
    rng = np.random.default_rng(12)
    buf = rng.integers(0, 256, 1024, dtype=np.uint8)
    for n in range(0, 601):
        for off in range(4):
            assert _half(emu, buf, off, n) == hashlib.sha512(buf[off:off + n].tobytes()).digest()[:32], (n, off)


def test_config5_lengths(emu):
    rng = np.random.default_rng(13)
    buf = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    for _ in range(400):
        n = int(np.exp(rng.uniform(np.log(100), np.log(4096))))
        off = int(rng.integers(0, buf.size - n))
        assert _half(emu, buf, off, n) == hashlib.sha512(buf[off:off + n].tobytes()).digest()[:32]


def test_block_from_window_matches_bytestream():
    """The hash kernels assemble each SHA-512 block from a 144-byte LDS window
    (block_from_window); on the host the same function must give ByteStream's
    blocks at every alignment and length, with and without the 4-byte prefix
    (the transaction-ID form "TXN\\0" || blob)."""
    import ctypes

    import numpy as np

    from tests.oracle_bind import load_hostemu
    emu = load_hostemu()
    rng = np.random.default_rng(9)
    buf = np.frombuffer(rng.bytes(6000), np.uint8).copy()
    base = buf.ctypes.data
    start = (16 - base % 16) % 16 + 32  # 16-byte aligned origin with room on both sides
    for off in range(start, start + 16):
        for ln in (0, 1, 3, 4, 5, 107, 108, 111, 112, 113, 127, 128, 129, 240, 256, 1000, 4100):
            assert emu.hostemu_window_blocks(buf.ctypes.data_as(ctypes.c_void_p), off, ln, 0, 0) == 0, (off, ln)
            assert emu.hostemu_window_blocks(buf.ctypes.data_as(ctypes.c_void_p), off, ln, 0x004E5854, 1) == 0, (off, ln)


def test_pair_rounds_equal_sha512(emu):
    """The long-row kernel's lane-pair rounds (stl_sha512.h pair_round_front /
    pair_round_back, both lanes emulated on the host): chaining the pair
    compression over padded messages gives hashlib's SHA-512, for lengths
    that cross block boundaries."""
    rng = np.random.default_rng(31)
    iv = [0x6a09e667f3bcc908, 0xbb67ae8584caa73b, 0x3c6ef372fe94f82b, 0xa54ff53a5f1d36f1,
          0x510e527fade682d1, 0x9b05688c2b3e6c1f, 0x1f83d9abfb41bd6b, 0x5be0cd19137e2179]
    for n in (0, 1, 111, 112, 127, 128, 239, 240, 1000, 4096):
        m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        pad = m + b"\x80" + b"\x00" * ((111 - n) % 128) + (8 * n).to_bytes(16, "big")
        assert len(pad) % 128 == 0
        for add64 in (1, 0):
            st = np.array(iv, dtype=np.uint64)
            for b in range(0, len(pad), 128):
                w = np.array([int.from_bytes(pad[b + 8 * j:b + 8 * j + 8], "big") for j in range(16)],
                             dtype=np.uint64)
                emu.hostemu_sha512_pair_compress(st.ctypes.data, w.ctypes.data, add64)
            got = b"".join(int(x).to_bytes(8, "big") for x in st)
            assert got == hashlib.sha512(m).digest(), (n, add64)
