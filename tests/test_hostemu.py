"""The device verify code (stellard_amd/csrc/stl_verify_core.h -- the exact
functions the gfx950 kernel runs) compiled for the host by the test harness
tests/native/hostemu.cpp: parity with the golden bits, and zero violations of
the 9x29-bit limb-bound discipline (stl_fe25519.h) on every golden input."""
import ctypes

import numpy as np
import pytest

from tests import oracle_bind


@pytest.fixture(scope="module")
def hostemu():
    return oracle_bind.load_hostemu()


def _run(lib, sig, msg, pk, policy):
    n = sig.shape[0]
    bm = np.zeros((n + 7) // 8, np.uint8)
    B = lambda a: np.ascontiguousarray(a).ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    viol = lib.hostemu_verify_batch(B(sig), B(msg), B(pk), n, B(bm), policy)
    return np.unpackbits(bm, bitorder="little")[:n].astype(bool), viol


@pytest.mark.parametrize("policy,key", [(0, "expected_sodium_1_0_18"), (1, "expected_stellard_1_0_0_unpinned")])
def test_hostemu_golden(hostemu, golden, policy, key):
    got, viol = _run(hostemu, golden["sig"], golden["msg"], golden["pk"], policy)
    assert viol == 0
    assert hostemu.hostemu_bound_checks() > 0
    assert np.array_equal(got, golden[key].astype(bool))


def test_hostemu_random_vs_oracle(hostemu, oracle):
    rng = np.random.default_rng(41)
    n = 400
    sig = np.zeros((n, 64), np.uint8)
    pk = np.zeros((n, 32), np.uint8)
    msg = rng.integers(0, 256, (n, 32), np.uint8)
    for i in range(n):
        p, sk = oracle.keypair(rng.bytes(32))
        pk[i] = np.frombuffer(p, np.uint8)
        sig[i] = np.frombuffer(oracle.sign(msg[i].tobytes(), sk), np.uint8)
        if i % 3 == 0:
            sig[i, rng.integers(64)] ^= 1 << rng.integers(8)
    got, viol = _run(hostemu, sig, msg, pk, 0)
    assert viol == 0
    assert np.array_equal(got, oracle.verify_batch(sig, msg, pk))
