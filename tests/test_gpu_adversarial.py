"""GPU tests of the adversarial classes at the boundary:

* the device's adversarial-row builder (stl_debug_sign_adversarial_device,
  the rows test_gpu_digests regenerates at 10M / 64M) equals the host's
  construction over libsodium (tests/datasets.py) byte for byte, and libstl's
  bits on those rows equal libsodium 1.0.18's (and the oracle's for the 1.0.0
  policy) class by class;
* the one reference-held expectation of the bare libsodium call: the
  RippleAddress_test S+L signature VERIFIES under the 1.0.0 predicate the
  reference pins (RippleAddress.cpp:838-845; Dockerfile:9-10) -- libstl's
  test-only raw mode (STL_DEBUG_RAW_PREDICATE) must accept it, and the
  composite (the product) must reject it.

Run on an MI355X:  python -u -m pytest tests -m gpu -x -v --timeout 120
"""
import hashlib

import numpy as np
import pytest

from tests import datasets, oracle_bind

pytestmark = pytest.mark.gpu

L = 2**252 + 27742317777372353535851937790883648493


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


def _device_rows(stl, torch, seeds, msgs, cls, param):
    t = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (seeds, msgs, cls, param.view(np.int32))]
    pk, sig, mo = stl.sign_adversarial_device(*t)
    return pk.cpu().numpy(), sig.cpu().numpy(), mo.cpu().numpy()


def test_device_builder_equals_host_construction(stl, torch_cuda, oracle):
    torch = torch_cuda
    lib = oracle_bind.load_sodium_ref()
    n = 30_000
    seeds, msgs, cls, param = datasets.chunk_plan(0x5EED0099, n, 0.5)
    assert set(np.unique(cls)) == set(range(datasets.NCLASSES + 1))
    pk_d, sig_d, msg_d = _device_rows(stl, torch, seeds, msgs, cls, param)
    honest = cls == 0
    if lib is not None:
        pk_h, sig_h = oracle_bind.sodium_sign_batch(lib, seeds, msgs, 16)
        group = datasets.sodium_group(lib)
    else:  # host construction over the oracle's signer and pure-Python group operations
        pk_h = np.zeros_like(pk_d)
        sig_h = np.zeros_like(sig_d)
        for i in range(n):
            p, sk = oracle.keypair(seeds[i].tobytes())
            pk_h[i] = np.frombuffer(p, np.uint8)
            sig_h[i] = np.frombuffer(oracle.sign(msgs[i].tobytes(), sk), np.uint8)
        group = datasets.python_group()
    msg_h = msgs.copy()
    assert np.array_equal(pk_d[honest], pk_h[honest]) and np.array_equal(sig_d[honest], sig_h[honest])
    datasets.mutate(seeds, msg_h, pk_h, sig_h, cls, param, group)
    for c in range(1, datasets.NCLASSES + 1):
        m = cls == c
        same = (pk_d[m] == pk_h[m]).all(axis=1) & (sig_d[m] == sig_h[m]).all(axis=1) & (msg_d[m] == msg_h[m]).all(axis=1)
        assert same.all(), (datasets.CLASSES[c], int((~same).sum()))
    # libstl's verdicts on every class: libsodium 1.0.18 (else the oracle), and the 1.0.0 policy vs the oracle
    words = stl.verify_batch_device(*[torch.from_numpy(a).cuda() for a in (sig_d, msg_d, pk_d)])
    torch.cuda.synchronize()
    got = stl.words_to_bool(words, n)
    exp = oracle_bind.sodium_verify_batch(lib, sig_d, msg_d, pk_d, 16) if lib is not None else \
        oracle.verify_batch(sig_d, msg_d, pk_d)
    assert np.array_equal(got, exp)
    assert got[honest].all() and not got[(cls >= 1) & (cls != 8)].any()  # only B8 (8 | k) can pass
    words = stl.verify_batch_device(*[torch.from_numpy(a).cuda() for a in (sig_d, msg_d, pk_d)],
                                    policy=stl.POLICY_STELLARD_1_0_0)
    torch.cuda.synchronize()
    got100 = stl.words_to_bool(words, n)
    assert np.array_equal(got100, oracle.verify_batch(sig_d, msg_d, pk_d, policy=1))
    # the 1.0.0 policy accepts what 1.0.18's extra checks reject: B6 keys of
    # order dividing k, B7 R = identity, B8 like 1.0.18
    assert got100[cls == 6].sum() > 0 and got100[cls == 7].sum() > 0


def test_raw_predicate_rippleaddress_kat(stl, oracle):
    """RippleAddress_test (RippleAddress.cpp:829-845): the masterpassphrase
    key signs the zero uint256; adding L to S must verify under the bare
    crypto_sign_verify_detached of the pinned libsodium 1.0.0, and fail
    stellard's composite."""
    from stellard_amd import _native as N
    seed = hashlib.sha512(b"masterpassphrase").digest()[:32]
    pk, sk = oracle.keypair(seed)
    msg = bytes(32)
    sig = oracle.sign(msg, sk)
    nc = sig[:32] + (int.from_bytes(sig[32:], "little") + L).to_bytes(32, "little")
    rows = [np.frombuffer(x, np.uint8).reshape(1, -1).repeat(70, axis=0) for x in (nc, msg, pk)]
    raw = N.STL_DEBUG_RAW_PREDICATE
    for flags, want in ((N.STL_POLICY_STELLARD_1_0_0 | raw, True),   # the reference's raw expectation
                        (N.STL_POLICY_STELLARD_1_0_0, False),         # stellard's composite
                        (N.STL_POLICY_SODIUM_1_0_18 | raw, False),    # 1.0.18 rejects S >= L itself
                        (N.STL_POLICY_SODIUM_1_0_18, False),
                        (N.STL_POLICY_STELLARD_1_0_0 | raw | N.STL_FULL_LENGTH, True),
                        (N.STL_POLICY_STELLARD_1_0_0 | raw | N.STL_ONE_LANE, True)):
        got = stl.verify_batch(*rows, policy=flags)
        assert got.all() == want and got.any() == want, hex(flags)
        assert oracle.verify_raw(nc, msg, pk, policy=flags & 1) == want or not (flags & raw)
    # the honest signature verifies in every mode
    rows = [np.frombuffer(x, np.uint8).reshape(1, -1) for x in (sig, msg, pk)]
    for flags in (0, 1, raw, 1 | raw):
        assert stl.verify_batch(*rows, policy=flags).all()
