"""In-tree build of every native artefact (no cmake, no JIT cache):

  stellard_amd/libstl.so         product: gfx950 kernels + C ABI (hipcc)
  tests/native/libhostemu.so     test harness: the device verify code compiled
                                 for the host (bound checks on)
  oracle/build/liboracle.so      test oracle: CPU restatement (make)
  oracle/_ref/libsodium_ref.so   test oracle: reference call path over libsodium

Usage: python -m stellard_amd.build [--product-only]
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "stellard_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")

PRODUCT_SRCS = ["stl_kernels.hip", "stl_api.cpp", "stl_batcher.cpp"]
PRODUCT_DEPS = PRODUCT_SRCS + ["stl_kernels.h", "stl_verify_core.h", "stl_fe25519.h", "stl_ge25519.h",
                               "stl_sc25519.h", "stl_sha512.h", "stl_base_table.h", "stl_lattice.h", "stl_txblob.h", "stl_sign.h",
                               os.path.join("..", "..", "include", "stl.h")]


def source_digest():
    """SHA-256 over the product's sources (PRODUCT_DEPS, in order): names the
    build a profile was taken on, and lets bench.py tell whether the committed
    profile summaries still describe the sources it runs."""
    import hashlib
    h = hashlib.sha256()
    for d in PRODUCT_DEPS:
        with open(os.path.join(CSRC, d), "rb") as f:
            h.update(os.path.basename(d).encode() + b"\0" + f.read())
    return h.hexdigest()


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, cwd=ROOT):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, cwd=cwd, check=True)


# per-object dependencies: the host sources see only the ABI header and the
# launcher declarations, so a host-side change does not recompile the kernels
# (about 100 s) -- the objects live in build/obj (git-ignored, never shipped)
HOST_DEPS = ["stl_kernels.h", os.path.join("..", "..", "include", "stl.h")]
OBJ_DIR = os.path.join(ROOT, "build", "obj")


def build_product(force=False, extra_flags=(), variant="variant"):
    out = os.path.join(ROOT, "stellard_amd", "libstl.so")
    deps = [os.path.join(CSRC, d) for d in PRODUCT_DEPS]
    if extra_flags:
        # variant builds (-D experiment switches): one command, nothing cached,
        # and never the product's path -- a variant written to libstl.so would
        # look newer than build/obj and survive the next default build (ADVICE
        # r5); load one with STL_LIB_PATH=build/ab/<variant>.so
        vout = os.path.join(ROOT, "build", "ab", variant + ".so")
        os.makedirs(os.path.dirname(vout), exist_ok=True)
        _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", *extra_flags,
              "-o", vout] + [os.path.join(CSRC, s) for s in PRODUCT_SRCS])
        return vout
    os.makedirs(OBJ_DIR, exist_ok=True)
    objs = []
    for src in PRODUCT_SRCS:
        obj = os.path.join(OBJ_DIR, src + ".o")
        sdeps = deps if src.endswith(".hip") else [os.path.join(CSRC, d) for d in [src] + HOST_DEPS]
        if force or _stale(obj, sdeps):
            _run([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", "-o", obj,
                  os.path.join(CSRC, src)])
        objs.append(obj)
    if force or _stale(out, objs):
        _run([HIPCC, f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", out] + objs)
    return out


def build_hostemu(force=False):
    out = os.path.join(ROOT, "tests", "native", "libhostemu.so")
    src = os.path.join(ROOT, "tests", "native", "hostemu.cpp")
    deps = [src] + [os.path.join(CSRC, d) for d in PRODUCT_DEPS]
    if force or _stale(out, deps):
        _run([HIPCC, "-O2", "-std=c++17", "-fPIC", "-shared", "-o", out, src])
    return out


def build_oracle():
    oracle = os.path.join(ROOT, "oracle")
    targets = ["build/liboracle.so"]
    # the libsodium harness only builds where libsodium's headers exist
    if os.path.exists("/opt/conda/include/sodium.h"):
        targets.append("_ref/libsodium_ref.so")
    _run(["make", "-s", "-C", oracle] + targets)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    force = "--force" in argv
    if "--product-only" in argv:
        build_product(force=force)
        return
    # the product and the host harness are independent single-threaded
    # compiles of the same device code: run them side by side
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=2) as ex:
        jobs = [ex.submit(build_product, force), ex.submit(build_hostemu, force)]
        for j in jobs:
            j.result()
    build_oracle()


if __name__ == "__main__":
    main()
