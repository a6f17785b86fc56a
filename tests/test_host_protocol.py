"""Host side of SerializedTransaction::checkSign (SerializedTransaction.cpp:
192-230) as mirrored by stellard_amd.verify.SignedTx / check_sign_batch:
SURVEY Appendix B class B12 (malformed lengths, missing TxnSignature) is a
host pre-reject that never reaches the GPU, the mSigGood / mSigBad cache
short-circuits, and the ledger-close pre-verify never records a reject.
These rows need no device: a call that reached libstl would raise ENODEV on
this GPU-less box."""
import pytest

from stellard_amd import verify as V

PRE = b"STX\x00" + bytes(109)


@pytest.mark.parametrize("pk,sig", [
    (bytes(33), bytes(64)),      # SigningPubKey not 32 bytes -> verifySignature throws
    (bytes(31), bytes(64)),
    (b"", bytes(64)),
    (bytes(32), bytes(63)),      # TxnSignature not 64 bytes
    (bytes(32), bytes(65)),
    (bytes(32), None),           # TxnSignature absent -> empty Blob
])
def test_b12_malformed_rejected_on_host(pk, sig):
    t = V.SignedTx(pk, sig, PRE)
    assert not t.well_formed()
    assert V.check_sign_batch([t]) == [False]
    assert t.sig_bad and not t.sig_good


def test_cache_short_circuits():
    good = V.SignedTx(bytes(32), bytes(64), PRE)
    good.set_good()
    bad = V.SignedTx(bytes(32), bytes(64), PRE)
    bad.sig_bad = True
    assert V.check_sign_batch([good, bad]) == [True, False]
    assert good.check_sign() is True


def test_good_only_never_records_reject():
    t = V.SignedTx(bytes(33), bytes(64), PRE)
    assert V.check_sign_batch([t], mark="good_only") == [False]
    assert not t.sig_bad and not t.sig_good


def test_well_formed_rows_go_to_the_device():
    """A well-formed row is sent to libstl; without a GPU that is an error,
    never a silent host verify."""
    t = V.SignedTx(bytes(32), bytes(64), PRE)
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from stellard_amd import _native as N
    with pytest.raises(N.StlError):
        V.check_sign_batch([t])
    assert not t.sig_good and not t.sig_bad
