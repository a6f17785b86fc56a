"""Sanitizer runs of the host-side code (the reference CI
ran under MALLOC_CHECK_=3 only, /root/reference/.travis.yml:45-49):

* AddressSanitizer + UndefinedBehaviorSanitizer (shift, bounds, null,
  alignment, vla-bound, return, unreachable, integer-divide-by-zero) over the
  host build of the
  device verify / blob code (tests/native/hostemu.cpp, the functions the
  gfx950 kernels run) and the C oracle, on the golden vectors and a
  serialized-transaction / validation corpus with mutations;
* ThreadSanitizer over the request aggregator (stl_batcher.cpp) with 6
  submitter threads, a flusher and the worker, through the ENODEV path and a
  verdict path (tests/native/tsan_batcher.cpp; ROCm's clang: GCC 11's TSan
  does not intercept pthread_cond_clockwait and reports false races).
No GPU code is sanitized (not available on this pool)."""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
OUT = os.path.join(NATIVE, "san")
CLANG = "/opt/rocm/lib/llvm/bin/clang"
CLANGXX = "/opt/rocm/lib/llvm/bin/clang++"
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
CSRC = os.path.join(ROOT, "stellard_amd", "csrc")


def _deps(*extra):
    # the host build compiles the __host__ __device__ headers only (hostemu.cpp
    # includes no .hip / .cpp of the product), so kernel-launcher edits do not
    # force the slow sanitizer rebuild
    d = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + \
        [os.path.join(ROOT, "include", "stl.h")]
    return d + [os.path.join(ROOT, "oracle", f) for f in ("stl_oracle.c", "stl_oracle_tx.c", "stl_oracle.h")] + \
        list(extra)


def _stale(out, deps):
    return not os.path.exists(out) or any(os.path.getmtime(p) > os.path.getmtime(out) for p in deps)


def _run(cmd):
    subprocess.run(cmd, check=True, cwd=ROOT)


def build_asan():
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "sanitize_main")
    main = os.path.join(NATIVE, "sanitize_main.cpp")
    if not _stale(exe, _deps(main, os.path.join(NATIVE, "hostemu.cpp"))):
        return exe
    # ASan + the UBSan checks that matter for this code (shifts, bounds, null,
    # alignment, ...).  -O1, no -g: the fully unrolled field products make a
    # full -fsanitize=undefined -O2 build take tens of minutes.
    san = ["-fsanitize=address,shift,bounds,null,alignment,vla-bound,return,unreachable,integer-divide-by-zero",
           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]
    objs = []
    for c in ("stl_oracle.c", "stl_oracle_tx.c"):
        o = os.path.join(OUT, c + ".o")
        _run([CLANG, "-c", "-O1", "-std=c11", "-D_GNU_SOURCE", *san, "-o", o, os.path.join(ROOT, "oracle", c)])
        objs.append(o)
    # host-only compile of the HIP headers' __host__ __device__ code; the GPU
    # side is not built (-fno-gpu-sanitize: nothing is sanitized on the device)
    o = os.path.join(OUT, "sanitize_main.o")
    _run([HIPCC, "-x", "hip", "--cuda-host-only", "-fno-gpu-sanitize", "-c", "-O1", "-std=c++17", *san,
          "-o", o, main])
    _run([HIPCC, "-fno-gpu-sanitize", *san, "-o", exe, o, *objs, "-lpthread"])
    return exe


def _vectors_file(golden, path):
    recs = np.concatenate([golden["sig"], golden["msg"], golden["pk"],
                           golden["expected_sodium_1_0_18"].reshape(-1, 1).astype(np.uint8),
                           golden["expected_stellard_1_0_0_unpinned"].reshape(-1, 1).astype(np.uint8)], axis=1)
    recs.astype(np.uint8).tofile(path)


def _blobs_file(oracle, path):
    from tests import txblob
    rng = np.random.default_rng(71)
    blobs = txblob.valid_corpus(oracle, 120, 72)
    blobs += [b for _, b, _ in txblob.special_cases(oracle)]
    keys = [oracle.keypair(rng.bytes(32)) for _ in range(3)]
    for i in range(60):
        pk, sk = keys[i % 3]
        b, _, _ = txblob.signed_validation(txblob.validation_fields(rng, pk), sk, oracle.sign)
        blobs.append(b)
    blobs += [txblob.mutate(rng, blobs[int(rng.integers(0, len(blobs)))]) for _ in range(400)]
    with open(path, "wb") as f:
        for b in blobs:
            f.write(struct.pack("<I", len(b)) + b)
    return len(blobs)


@pytest.mark.timeout(900)
def test_asan_ubsan_device_code_and_oracle(golden, oracle, tmp_path):
    exe = build_asan()
    vec, blb = str(tmp_path / "vectors.bin"), str(tmp_path / "blobs.bin")
    _vectors_file(golden, vec)
    nb = _blobs_file(oracle, blb)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([exe, vec, blb], capture_output=True, text=True, timeout=840, env=env)
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert f"vectors {golden['sig'].shape[0]} blobs {nb} compared" in r.stdout
    assert r.stdout.strip().endswith("disagreements 0")
    compared = int(r.stdout.split("compared")[1].split()[0])
    assert compared > 300


def build_tsan():
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "tsan_batcher")
    src = os.path.join(NATIVE, "tsan_batcher.cpp")
    if _stale(exe, [src, os.path.join(CSRC, "stl_batcher.cpp"), os.path.join(ROOT, "include", "stl.h")]):
        _run([CLANGXX, "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread", "-o", exe, src])
    return exe


@pytest.mark.parametrize("mode", ["enodev", "bits"])
def test_tsan_batcher(mode):
    exe = build_tsan()
    r = subprocess.run([exe, mode], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1"))
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]
    assert "submitted=9000 completed=9000" in r.stdout and "bad=0" in r.stdout
