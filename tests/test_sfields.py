"""The serialization tables of the blob path pinned to the reference's own text
(SURVEY 8 rows f1 / f4).

tests/golden/sfields.json is generated from the reference's source files by
tests/golden/make_sfields.py (SerializeDeclarations.h:33-205 field codes,
FieldNames.cpp:49-51 non-signing fields, TxFormats.h TxType enum,
TxFormats.cpp:22-130 templates without the commented-out Contract formats,
SerializedValidation.cpp:134-159).  Three restatements must equal it:

  device   stellard_amd/csrc/stl_txblob.h -- declared_names, tx_field_bit,
           tx_format, validation_field, non_signing_field -- through its host
           build (tests/native/libhostemu.so)
  oracle   oracle/stl_oracle_tx.c -- field_declared, kCommonFields /
           kTxFormats (order and SOE flags), kValidationFields, non_signing
  python   tests/txblob.py's named fields and NON_SIGNING

and a deliberately edited template or field makes the comparison fail
(test_comparison_catches_edits)."""
import copy
import ctypes
import json
import os

import pytest

from tests import txblob as T
from tests.oracle_bind import load_hostemu, load_oracle

HERE = os.path.dirname(os.path.abspath(__file__))
SOE_FLAG = {"SOE_REQUIRED": 0, "SOE_OPTIONAL": 1, "SOE_DEFAULT": 2}


@pytest.fixture(scope="module")
def ref():
    with open(os.path.join(HERE, "golden", "sfields.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def emu():
    lib = load_hostemu()
    lib.hostemu_tx_field_bit.restype = ctypes.c_int
    lib.hostemu_tx_field_bit.argtypes = [ctypes.c_uint32]
    lib.hostemu_tx_format.restype = ctypes.c_int
    lib.hostemu_tx_format.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    lib.hostemu_declared_names.restype = ctypes.c_uint64
    lib.hostemu_declared_names.argtypes = [ctypes.c_uint32]
    lib.hostemu_validation_field.restype = ctypes.c_int
    lib.hostemu_validation_field.argtypes = [ctypes.c_uint32]
    lib.hostemu_non_signing_field.restype = ctypes.c_int
    lib.hostemu_non_signing_field.argtypes = [ctypes.c_uint32]
    return lib


@pytest.fixture(scope="module")
def orc():
    lib = load_oracle().lib
    lib.oracle_table_declared.restype = ctypes.c_int
    lib.oracle_table_declared.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.oracle_table_non_signing.restype = ctypes.c_int
    lib.oracle_table_non_signing.argtypes = [ctypes.c_uint32]
    lib.oracle_table_tx_format.restype = ctypes.c_int
    lib.oracle_table_tx_format.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    lib.oracle_table_validation.restype = ctypes.c_int
    lib.oracle_table_validation.argtypes = [ctypes.c_void_p, ctypes.c_int]
    return lib


# ---------------------------------------------------------------- expected values from the JSON
def codes(ref):
    return {f["name"]: f["code"] for f in ref["fields"]}


def all_type_codes():
    return list(range(0, 21))


# ---------------------------------------------------------------- the restatements, read out
def device_tables(emu, ref):
    """What the device pass uses, in the JSON's vocabulary."""
    code = codes(ref)
    declared = {t: emu.hostemu_declared_names(t) for t in all_type_codes()}
    bit = {name: emu.hostemu_tx_field_bit(c) for name, c in code.items()}
    formats = {}
    for tt in list(ref["tx_types"].values()) + [11, 99, 102, 0xFFFF]:
        if tt < 0:
            continue
        a, r = ctypes.c_uint64(0), ctypes.c_uint64(0)
        if emu.hostemu_tx_format(tt, ctypes.byref(a), ctypes.byref(r)):
            formats[tt] = (a.value, r.value)
    return {"declared": declared, "bit": bit, "formats": formats,
            "validation": {n for n, c in code.items() if emu.hostemu_validation_field(c)},
            "non_signing": {n for n, c in code.items() if emu.hostemu_non_signing_field(c)}}


def oracle_tables(orc, ref):
    code = codes(ref)
    declared = {t: sum(1 << n for n in range(1, 64) if orc.oracle_table_declared(t, n)) for t in all_type_codes()}
    formats = {}
    cs, fl = (ctypes.c_uint32 * 64)(), (ctypes.c_int * 64)()
    for tt in list(ref["tx_types"].values()) + [11, 99, 102, 0xFFFF]:
        if tt < 0:
            continue
        k = orc.oracle_table_tx_format(tt, cs, fl, 64)
        if k >= 0:
            formats[tt] = [(cs[i], fl[i]) for i in range(k)]
    vc = (ctypes.c_uint32 * 64)()
    nv = orc.oracle_table_validation(vc, 64)
    by_code = {c: n for n, c in code.items()}
    return {"declared": declared, "formats": formats, "validation": {by_code.get(vc[i]) for i in range(nv)},
            "non_signing": {n for n, c in code.items() if orc.oracle_table_non_signing(c)}}


# ---------------------------------------------------------------- comparisons (return mismatches)
def compare_device(dev, ref):
    bad = []
    code = codes(ref)
    want_decl = {t: 0 for t in all_type_codes()}
    for f in ref["fields"]:
        want_decl[f["type_code"]] |= 1 << f["index"]
    for t in all_type_codes():
        if dev["declared"][t] != want_decl[t]:
            bad.append(("declared_names", t, hex(dev["declared"][t]), hex(want_decl[t])))
    in_tx = {n for n, _ in ref["common_fields"]} | {n for v in ref["tx_formats"].values() for n, _ in v["fields"]}
    bits = {}
    for n in code:
        b = dev["bit"][n]
        if (b >= 0) != (n in in_tx):
            bad.append(("tx_field_bit", n, b))
        if b >= 0:
            if b in bits:
                bad.append(("tx_field_bit shared", n, bits[b]))
            bits[b] = n
    by_type = {v["type"]: v for v in ref["tx_formats"].values()}
    for tt in set(dev["formats"]) | set(by_type):
        if tt not in by_type or tt not in dev["formats"]:
            bad.append(("tx_format presence", tt))
            continue
        els = ref["common_fields"] + by_type[tt]["fields"]
        allowed = sum(1 << dev["bit"][n] for n, _ in els if dev["bit"][n] >= 0)
        required = sum(1 << dev["bit"][n] for n, s in els if s == "SOE_REQUIRED" and dev["bit"][n] >= 0)
        if dev["formats"][tt] != (allowed, required):
            bad.append(("tx_format", tt, [hex(x) for x in dev["formats"][tt]], hex(allowed), hex(required)))
    if dev["validation"] != {n for n, _ in ref["validation"]}:
        bad.append(("validation_field", sorted(dev["validation"] ^ {n for n, _ in ref["validation"]})))
    if dev["non_signing"] != set(ref["non_signing"]):
        bad.append(("non_signing_field", sorted(dev["non_signing"])))
    return bad


def compare_oracle(orc_t, ref):
    bad = []
    code = codes(ref)
    want_decl = {t: 0 for t in all_type_codes()}
    for f in ref["fields"]:
        want_decl[f["type_code"]] |= 1 << f["index"]
    for t in all_type_codes():
        if orc_t["declared"][t] != want_decl[t]:
            bad.append(("field_declared", t))
    by_type = {v["type"]: v for v in ref["tx_formats"].values()}
    if set(orc_t["formats"]) != set(by_type):
        bad.append(("tx format types", sorted(set(orc_t["formats"]) ^ set(by_type))))
    for tt, v in by_type.items():
        want = [(code[n], SOE_FLAG[s]) for n, s in ref["common_fields"] + v["fields"]]
        if orc_t["formats"].get(tt) != want:
            bad.append(("kTxFormats", tt))
    if orc_t["validation"] != {n for n, _ in ref["validation"]}:
        bad.append(("kValidationFields",))
    if orc_t["non_signing"] != set(ref["non_signing"]):
        bad.append(("non_signing",))
    return bad


def compare_python(ref):
    bad = []
    types = ref["types"]
    for tname, t in types.items():
        if getattr(T, tname, t) != t:
            bad.append(("type id", tname))
    fields = {f["name"]: (f["type_code"], f["index"]) for f in ref["fields"]}
    named = {k: v for k, v in vars(T).items() if isinstance(v, tuple) and len(v) == 2 and k in fields}
    assert len(named) >= 40  # tests/txblob.py names most of the fields it writes
    for k, v in named.items():
        if v != fields[k]:
            bad.append(("txblob field", k, v, fields[k]))
    if T.NON_SIGNING != {fields[n] for n in ref["non_signing"]}:
        bad.append(("NON_SIGNING",))
    return bad


# ---------------------------------------------------------------- tests
def test_json_is_the_reference_text(ref):
    """Sanity of the generated file: 14 types, 117 fields with unique codes,
    the ten live TxFormats (the /* */ Contract formats absent), the 12-field
    validation template."""
    assert len(ref["types"]) == 14
    assert len({f["code"] for f in ref["fields"]}) == len(ref["fields"]) == 117
    assert sorted(v["type"] for v in ref["tx_formats"].values()) == [0, 1, 3, 4, 5, 7, 8, 20, 100, 101]
    assert "Contract" not in ref["tx_formats"] and "RemoveContract" not in ref["tx_formats"]
    assert len(ref["common_fields"]) == 13 and len(ref["validation"]) == 12


def test_device_tables_equal_reference(emu, ref):
    assert compare_device(device_tables(emu, ref), ref) == []


def test_oracle_tables_equal_reference(orc, ref):
    assert compare_oracle(oracle_tables(orc, ref), ref) == []


def test_python_serializer_equals_reference(ref):
    assert compare_python(ref) == []


def test_comparison_catches_edits(emu, orc, ref):
    """A one-bit edit of the expected tables -- a template flag, a template
    member, a field index, the non-signing set -- is reported by every
    comparison it touches (the pin has teeth)."""
    dev, ora = device_tables(emu, ref), oracle_tables(orc, ref)
    edits = []
    e = copy.deepcopy(ref)
    e["tx_formats"]["Payment"]["fields"][2][1] = "SOE_REQUIRED"  # SendMax required
    edits.append(e)
    e = copy.deepcopy(ref)
    e["tx_formats"]["OfferCancel"]["fields"].append(["Expiration", "SOE_OPTIONAL"])
    edits.append(e)
    e = copy.deepcopy(ref)
    e["common_fields"] = [x for x in e["common_fields"] if x[0] != "OperationLimit"]
    edits.append(e)
    for e in edits:
        assert compare_device(dev, e), "device comparison missed an edited template"
        assert compare_oracle(ora, e), "oracle comparison missed an edited template"
    e = copy.deepcopy(ref)
    next(f for f in e["fields"] if f["name"] == "DestinationTag")["index"] = 15
    for f in e["fields"]:
        f["code"] = (f["type_code"] << 16) | f["index"]
    assert compare_device(dev, e) and compare_oracle(ora, e) and compare_python(e)
    e = copy.deepcopy(ref)
    e["non_signing"] = ["TxnSignature", "Signature"]
    assert compare_device(dev, e) and compare_oracle(ora, e) and compare_python(e)
