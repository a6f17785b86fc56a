"""examples/ledger_close.cpp: libstl used from C++ the way stellard would use
it (stl.h + libstl.so, INTEGRATION.md sections 2, 4, 4b), built with g++ in
the test.  On CPU the example must compile, see STL_ENODEV and leave every
transaction to the serial path; on the GPU its accept bitmap equals the
oracle's and the six aggregator workers' verdicts equal the batch's."""
import hashlib
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "examples", "ledger_close.cpp")
EXE = os.path.join(ROOT, "examples", "ledger_close")


def build():
    lib = os.path.join(ROOT, "stellard_amd")
    if os.path.exists(EXE) and os.path.getmtime(EXE) > max(os.path.getmtime(SRC),
                                                           os.path.getmtime(os.path.join(ROOT, "include", "stl.h"))):
        return EXE
    subprocess.run([shutil.which("g++") or "g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror",
                    "-I", os.path.join(ROOT, "include"), SRC, "-L", lib, "-lstl", f"-Wl,-rpath,{lib}",
                    "-Wl,-rpath,/opt/rocm/lib", "-L/opt/rocm/lib", "-lamdhip64", "-pthread", "-o", EXE],
                   check=True)
    return EXE


def write_set(path, oracle, n, seed):
    rng = np.random.default_rng(seed)
    keys = [oracle.keypair(rng.bytes(32)) for _ in range(16)]
    rows = []
    with open(path, "wb") as f:
        f.write(struct.pack("<I", n))
        for i in range(n):
            pk, sk = keys[i % 16]
            pre = b"STX\x00" + rng.bytes(int(rng.integers(100, 700)))
            h = hashlib.sha512(pre).digest()[:32]
            sig = bytearray(oracle.sign(h, sk))
            if rng.random() < 0.25:
                sig[int(rng.integers(0, 64))] ^= 1 << int(rng.integers(0, 8))
            f.write(struct.pack("<I", len(pre)) + pre + h + bytes(sig) + pk)
            rows.append((pre, bytes(sig), pk))
    return rows


def run(tmp_path, oracle, n=1500):
    exe = build()
    data = str(tmp_path / "set.bin")
    rows = write_set(data, oracle, n, 5)
    r = subprocess.run([exe, data], capture_output=True, text=True, timeout=240)
    return r, rows


def test_example_builds_and_falls_back_without_gpu(tmp_path, oracle):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: see the gpu test")
    r, rows = run(tmp_path, oracle, n=50)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "stl_init -19" in r.stdout and "batch rc -19" in r.stdout
    bitmap = [l for l in r.stdout.splitlines() if l.startswith("bitmap ")][0].split()[1]
    assert bitmap == "0" * 50  # nothing pre-marked: the serial checkSign decides every one


@pytest.mark.gpu
def test_example_on_gpu(tmp_path, oracle):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r, rows = run(tmp_path, oracle)
    assert r.returncode == 0, r.stdout + r.stderr
    out = r.stdout
    bitmap = [l for l in out.splitlines() if l.startswith("bitmap ")][0].split()[1]
    got = np.array([c == "1" for c in bitmap])
    sig = np.frombuffer(b"".join(s for _, s, _ in rows), np.uint8).reshape(-1, 64)
    pk = np.frombuffer(b"".join(p for _, _, p in rows), np.uint8).reshape(-1, 32)
    exp = oracle.tx_verify_batch([p for p, _, _ in rows], sig, pk)
    assert np.array_equal(got, exp)
    assert "batch rc 0" in out and "batcher asked 600 agree 600 errors 0" in out, out
