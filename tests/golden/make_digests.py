#!/usr/bin/env python3
"""Generates tests/golden/bitmap_digests.json: SHA-256 digests of the accept
bitmaps libsodium 1.0.18 gives the seeded datasets of BASELINE.json configs 2,
4 and 3 (tests/datasets.py), with the digests of the inputs.

Run here (the build container: libsodium at /opt/conda/lib), never on the GPU
box.  Signing and verification both go through oracle/_ref/libsodium_ref.so
(crypto_sign_seed_keypair + crypto_sign_detached, and the reference's
verifySignature = crypto_sign_verify_detached && S < L).

    python tests/golden/make_digests.py [config2 config4 config3]
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests import datasets, oracle_bind  # noqa: E402


def main(names):
    lib = oracle_bind.load_sodium_ref()
    assert lib is not None, "needs libsodium"
    threads = os.cpu_count() or 8
    out = {}
    if os.path.exists(datasets.DIGESTS):
        with open(datasets.DIGESTS) as f:
            out = json.load(f)
    group = datasets.sodium_group(lib)
    for name in names:
        t0 = time.time()
        dg = datasets.Digest()
        classes, keys = {}, []

        def make(seeds, msgs, cls, param):
            pk, sig = oracle_bind.sodium_sign_batch(lib, seeds, msgs, threads)
            msgs = msgs.copy()
            datasets.mutate(seeds, msgs, pk, sig, cls, param, group)
            return pk, sig, msgs

        for c0, seed, n, frac in datasets.chunks(name):
            sig, msg, pk, cls = datasets.chunk(seed, n, frac, make)
            bits = oracle_bind.sodium_verify_batch(lib, sig, msg, pk, threads)
            dg.add(sig, msg, pk, bits)
            for k, v in datasets.class_counts(cls).items():
                classes[k] = classes.get(k, 0) + v
            adv = np.nonzero(cls)[0]
            keys.append(datasets.row_keys(sig[adv], msg[adv], pk[adv]))
            print(f"{name}: rows {c0 + n} accepted {dg.accepted} ({time.time() - t0:.0f} s)", flush=True)
        keys = np.concatenate(keys) if keys else np.zeros(0, "S16")
        out[name] = dict(dg.result(), **datasets.CONFIGS[name], adversarial_rows_by_class=classes,
                         adversarial_rows_distinct=int(np.unique(keys).size),
                         construction="each adversarial row mutated from its own honest row, classes B1-B11 "
                                      "evenly (tests/datasets.py)",
                         expected_from=f"libsodium {lib.ref_sodium_version().decode()} "
                                       "crypto_sign_verify_detached && S < L")
        with open(datasets.DIGESTS, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:] or ["config2", "config4", "config3"])
