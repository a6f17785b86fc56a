"""Seeded synthetic datasets of BASELINE.json configs 2-4 (test
infrastructure): the same bytes whoever signs them, because RFC 8032 signing
is deterministic -- libsodium here (tests/golden/make_digests.py, which commits
SHA-256 digests of libsodium's expected accept bitmaps) and the GPU signer on
the box (tests/test_gpu_digests.py, which checks libstl's bitmaps against
those digests).

  config 2   1,048,576 valid signatures, seed 0x5EED0002 (= bench.py rank 0)
  config 4   10,000,000 signatures, 2 % of rows replaced by golden adversarial
             rows (every SURVEY Appendix-B class), chunks of 2,000,000 with
             seed 0x5EED0004 + chunk offset
  config 3   67,108,864 signatures, same construction, chunks of 4,194,304
             with seed 0x5EED0003 + chunk offset

Row construction (per chunk): rng = default_rng(seed); seeds = 32 random
bytes per row, msgs = 32 random bytes per row; (pk, sig) = sign(seeds, msgs);
rows = rng.choice(n, int(n * frac), replace=False) are replaced by golden
rows rng.integers(0, pool) of the non-valid classes -- the construction
tools/report_configs.py used for the round-1 64M run.
"""
import hashlib
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CONFIGS = {
    "config2": {"n": 1 << 20, "chunk": 1 << 20, "seed": 0x5EED0002, "frac": 0.0},
    "config4": {"n": 10_000_000, "chunk": 2_000_000, "seed": 0x5EED0004, "frac": 0.02},
    "config3": {"n": 1 << 26, "chunk": 1 << 22, "seed": 0x5EED0003, "frac": 0.02},
}

DIGESTS = os.path.join(ROOT, "tests", "golden", "bitmap_digests.json")


def adversarial_pool():
    g = np.load(os.path.join(ROOT, "tests", "golden", "ed25519_golden.npz"), allow_pickle=False)
    names = [str(x) for x in g["class_names"]]
    idx = np.nonzero(g["cls"] != names.index("valid"))[0]
    return g["sig"][idx], g["msg"][idx], g["pk"][idx], g["cls"][idx], names


def chunk(seed, n, frac, sign, pool=None):
    """One chunk: (sig, msg, pk, class counts).  sign(seeds, msgs) -> (pk, sig)
    as uint8 numpy arrays."""
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pk, sig = sign(seeds, msgs)
    pk, sig = np.array(pk, np.uint8, copy=True), np.array(sig, np.uint8, copy=True)
    classes = {}
    if frac > 0:
        asig, amsg, apk, acls, names = pool if pool is not None else adversarial_pool()
        rows = rng.choice(n, int(n * frac), replace=False)
        pick = rng.integers(0, asig.shape[0], rows.size)
        sig[rows], msgs[rows], pk[rows] = asig[pick], amsg[pick], apk[pick]
        classes = {names[c]: int((acls[pick] == c).sum()) for c in np.unique(acls[pick])}
    return sig, msgs, pk, classes


def chunks(name):
    c = CONFIGS[name]
    for c0 in range(0, c["n"], c["chunk"]):
        yield c0, c["seed"] + (c0 if c["frac"] > 0 else 0), min(c["chunk"], c["n"] - c0), c["frac"]


class Digest:
    """Running SHA-256 of the packed accept bitmap (LSB first, chunk after
    chunk -- every chunk is a multiple of 8 rows) and of the input rows."""

    def __init__(self):
        self.bits = hashlib.sha256()
        self.inputs = hashlib.sha256()
        self.rows = 0
        self.accepted = 0

    def add(self, sig, msg, pk, bits):
        assert bits.shape[0] % 8 == 0 or self.rows == 0
        self.inputs.update(np.ascontiguousarray(sig).tobytes())
        self.inputs.update(np.ascontiguousarray(msg).tobytes())
        self.inputs.update(np.ascontiguousarray(pk).tobytes())
        self.bits.update(np.packbits(np.asarray(bits, bool), bitorder="little").tobytes())
        self.rows += bits.shape[0]
        self.accepted += int(np.count_nonzero(bits))

    def result(self):
        return {"rows": self.rows, "accepted": self.accepted, "bitmap_sha256": self.bits.hexdigest(),
                "inputs_sha256": self.inputs.hexdigest()}
