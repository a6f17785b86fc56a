#!/usr/bin/env python3
"""Generates tests/golden/sfields.json from the reference's own source text --
the serialization tables the blob path restates:

  src/ripple_data/protocol/SerializeDeclarations.h   TYPE / FIELD lines: every
                                                      (type, index, name)
  src/ripple_data/protocol/FieldNames.cpp             initFields: the fields
                                                      marked notSigningField
  src/ripple_data/protocol/TxFormats.h                the TxType enum
  src/ripple_data/protocol/TxFormats.cpp              each add(...) template and
                                                      addCommonFields, with the
                                                      /* */-commented formats
                                                      (Contract, RemoveContract)
                                                      left out as the compiler
                                                      leaves them out
  src/ripple_app/ledger/SerializedValidation.cpp      getFormat: the validation
                                                      template

The files are read as text and parsed with regular expressions; nothing of the
reference is executed or copied, only the table VALUES land in the JSON (with
the SHA-256 of every source file read).  Run here, in the build container
(/root/reference exists only here):

    python tests/golden/make_sfields.py
"""
import hashlib
import json
import os
import re
import sys

REF = os.environ.get("STL_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "sfields.json")

FILES = {
    "declarations": "src/ripple_data/protocol/SerializeDeclarations.h",
    "field_names": "src/ripple_data/protocol/FieldNames.cpp",
    "tx_types": "src/ripple_data/protocol/TxFormats.h",
    "tx_formats": "src/ripple_data/protocol/TxFormats.cpp",
    "validation": "src/ripple_app/ledger/SerializedValidation.cpp",
}


def strip_comments(text):
    """Remove /* ... */ blocks and // line comments (as the C preprocessor
    does; no string literal in these files contains either)."""
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    return re.sub(r"//[^\n]*", "", text)


def read(key):
    with open(os.path.join(REF, FILES[key]), "rb") as f:
        raw = f.read()
    return raw.decode("utf-8", "replace"), hashlib.sha256(raw).hexdigest()


def parse_declarations(text):
    body = strip_comments(text)
    types = {m.group(2): int(m.group(3)) for m in
             re.finditer(r"^\s*TYPE\s*\(\s*(\w+)\s*,\s*(\w+)\s*,\s*(\d+)\s*\)", body, re.M)}
    fields = []
    for m in re.finditer(r"^\s*FIELD\s*\(\s*(\w+)\s*,\s*(\w+)\s*,\s*(\d+)\s*\)", body, re.M):
        name, tname, idx = m.group(1), m.group(2), int(m.group(3))
        t = types[tname]
        fields.append({"name": name, "type": tname, "type_code": t, "index": idx, "code": (t << 16) | idx})
    return types, fields


def parse_non_signing(text):
    body = strip_comments(text)
    m = re.search(r"initFields\s*\(\s*\)\s*\{(.*?)\n\}", body, re.S)
    return sorted(set(re.findall(r"sf(\w+)\s*\.\s*notSigningField\s*\(\s*\)", m.group(1))))


def parse_tx_types(text):
    body = strip_comments(text)
    m = re.search(r"enum\s+TxType\s*\{(.*?)\}", body, re.S)
    return {k: int(v) for k, v in re.findall(r"(tt\w+)\s*=\s*(-?\d+)", m.group(1))}


SOE = r"SOElement\s*\(\s*sf(\w+)\s*,\s*(SOE_\w+)\s*\)"


def parse_tx_formats(text, tx_types):
    body = strip_comments(text)
    formats = {}
    for m in re.finditer(r"\badd\s*\(\s*\"(\w+)\"\s*,\s*(tt\w+)\s*\)(.*?);", body, re.S):
        formats[m.group(1)] = {"tx_type": m.group(2), "type": tx_types[m.group(2)],
                               "fields": [[f, s] for f, s in re.findall(SOE, m.group(3))]}
    m = re.search(r"addCommonFields\s*\([^)]*\)\s*\{(.*?)\}", body, re.S)
    common = [[f, s] for f, s in re.findall(SOE, m.group(1))]
    return formats, common


def parse_validation(text):
    body = strip_comments(text)
    m = re.search(r"getFormat\s*\(\s*\)\s*\{(.*?)static\s+FormatHolder", body, re.S)
    return [[f, s] for f, s in re.findall(r"push_back\s*\(\s*" + SOE + r"\s*\)", m.group(1))]


def main():
    src = {}
    texts = {}
    for k, path in FILES.items():
        texts[k], src[path] = read(k)
    types, fields = parse_declarations(texts["declarations"])
    tx_types = parse_tx_types(texts["tx_types"])
    formats, common = parse_tx_formats(texts["tx_formats"], tx_types)
    doc = {
        "generated_by": "tests/golden/make_sfields.py (regular expressions over the reference's source text)",
        "sources_sha256": src,
        "types": types,
        "fields": fields,
        "non_signing": parse_non_signing(texts["field_names"]),
        "tx_types": tx_types,
        "common_fields": common,
        "tx_formats": formats,
        "validation": parse_validation(texts["validation"]),
    }
    names = {f["name"] for f in fields}
    for f, _ in common + [x for v in formats.values() for x in v["fields"]] + doc["validation"]:
        assert f in names, f
    assert len(fields) == len(names), "duplicate field names"
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print(f"{len(fields)} fields, {len(formats)} transaction formats, non-signing {doc['non_signing']} -> {OUT}")


if __name__ == "__main__":
    sys.exit(main())
