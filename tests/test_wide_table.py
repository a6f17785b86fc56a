"""The wide base tables of the half-size check ([e]B with radix-2^16 digits,
stl_verify_core.h wide_entry; built on the device at stl_init by
wide_table_kernel, on the host by the same function): rows 1..128 equal the
committed 128-entry tables (tools/gen_base_table.py, independent Python
arithmetic), row 0 is the identity, and sampled rows up to 32768 equal j*B
and j*2^128*B computed in Python."""
import ctypes

import numpy as np
import pytest

from tests.oracle_bind import load_hostemu

P = 2**255 - 19
D = (-121665 * pow(121666, P - 2, P)) % P
L = 2**252 + 27742317777372353535851937790883648493


def ed_add(a, b):
    x1, y1 = a
    x2, y2 = b
    t = D * x1 * x2 * y1 * y2 % P
    x3 = (x1 * y2 + x2 * y1) * pow(1 + t, P - 2, P) % P
    y3 = (y1 * y2 + x1 * x2) * pow(1 - t, P - 2, P) % P
    return x3, y3


def ed_mul(k, a):
    r = (0, 1)
    while k:
        if k & 1:
            r = ed_add(r, a)
        a = ed_add(a, a)
        k >>= 1
    return r


BY = 4 * pow(5, P - 2, P) % P
BX = None


def base_point():
    global BX
    if BX is None:
        u = (BY * BY - 1) % P
        v = (D * BY * BY + 1) % P
        x = pow(u * pow(v, P - 2, P), (P + 3) // 8, P)
        if (x * x - u * pow(v, P - 2, P)) % P != 0:
            x = x * pow(2, (P - 1) // 4, P) % P
        if x & 1:
            x = P - x
        BX = x
    return BX, BY


def limbs_to_int(words):
    return sum(int(w) << (29 * i) for i, w in enumerate(words[:9]))


def row(emu, which, j):
    out = (ctypes.c_uint32 * 28)()
    emu.hostemu_wide_row(which, j, out)
    return list(out)


@pytest.fixture(scope="module")
def emu():
    return load_hostemu()


def test_identity_row(emu):
    for which in (0, 1):
        r = row(emu, which, 0)
        assert limbs_to_int(r[0:9]) == 1 and limbs_to_int(r[9:18]) == 1 and limbs_to_int(r[18:27]) == 0


@pytest.mark.parametrize("which", [0, 1])
def test_rows_match_committed_tables(emu, which):
    import re
    text = open(__file__.replace("tests/test_wide_table.py", "stellard_amd/csrc/stl_base_table.h")).read()
    host = text[text.index("kBaseNielsHost"):]
    nums = [int(x, 16) for x in re.findall(r"0x([0-9a-fA-F]+)u?", host)][: 2 * 128 * 28]
    ref = np.array(nums, np.uint64).reshape(2, 128, 28)
    for j in (1, 2, 3, 64, 127, 128):
        assert row(emu, which, j) == [int(v) for v in ref[which, j - 1]], j


@pytest.mark.parametrize("j", [129, 255, 256, 1000, 4097, 12345, 32767, 32768])
def test_rows_match_python(emu, j):
    B = base_point()
    B128 = ed_mul(2**128, B)
    for which, Pt in ((0, B), (1, B128)):
        x, y = ed_mul(j, Pt)
        r = row(emu, which, j)
        assert limbs_to_int(r[0:9]) == (y + x) % P
        assert limbs_to_int(r[9:18]) == (y - x) % P
        assert limbs_to_int(r[18:27]) == 2 * D * x * y % P
        assert max(r[:27]) < 2**29 and r[27] == 0


def _encode(pt):
    x, y = pt
    return (y | ((x & 1) << 255)).to_bytes(32, "little")


@pytest.mark.parametrize("m", [5, 2**200 + 12345, L - 1])
def test_wide_key_table_two_stages(emu, m):
    """Round 6: the wide per-key tables j*(-A), j = 0..136, are built in two
    stages (24 entries by double-and-add, the other 113 as one addition of two
    of them: key_table_wide_base_kernel / key_table_wide_pair_kernel).  On the
    host build of the same functions every entry equals the one-stage
    double-and-add of j and -j*m*B computed in Python, for keys A = m*B."""
    B = base_point()
    A = ed_mul(m, B)
    two = (ctypes.c_uint8 * (137 * 64))()
    one = (ctypes.c_uint8 * (137 * 64))()
    assert emu.hostemu_wide_key_table(_encode(A), two, one) == 1
    assert bytes(two) == bytes(one)
    for j in (0, 1, 15, 16, 17, 31, 33, 100, 128, 129, 136):
        x, y = ed_mul(j * m % L, B) if j else (0, 1)
        want = ((P - x) % P).to_bytes(32, "little") + y.to_bytes(32, "little")
        assert bytes(two[64 * j:64 * j + 64]) == want, j


def test_wide_key_table_small_order_key(emu):
    """A key of order 8 (torsion, golden class B6-B8 material): the two-stage
    table equals the double-and-add one for every j (the additions meet equal
    and opposite points and the identity -- the complete formula's cases)."""
    # an order-8 point: x^2 = ... pick the encoding from the small-order list
    enc = bytes.fromhex("c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a")
    two = (ctypes.c_uint8 * (137 * 64))()
    one = (ctypes.c_uint8 * (137 * 64))()
    assert emu.hostemu_wide_key_table(enc, two, one) == 1
    assert bytes(two) == bytes(one)
