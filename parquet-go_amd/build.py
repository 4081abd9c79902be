"""In-tree build of the native libraries (no JIT cache: the .so files travel with the repo).

  libpqhip.so  — product: HIP kernels for gfx950 + host page walker + C-ABI (include/pqhip.h)
  libpqgen.so  — tooling: reference-writer-shaped file generator (csrc/tools/pqgen.h)

Usage:  python parquet-go_amd/build.py [--force]
"""
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
INCLUDE = os.path.join(ROOT, "include")

HOST_SRCS = ["host/codec.cpp", "host/file_reader.cpp"]
HIP_SRCS = ["kernels/decode.hip", "host/batch.hip"]
GEN_SRCS = ["tools/pqgen.cpp", "host/codec.cpp"]
HEADERS = sorted(os.path.relpath(os.path.join(d, f), CSRC) for d, _, fs in os.walk(CSRC) for f in fs
                 if f.endswith(".h"))

ARCH = os.environ.get("PQH_OFFLOAD_ARCH", "gfx950")
# PQH_SANITIZE=1 (or --sanitize): ASan + UBSan variants of the host parsers -- codec.cpp and
# file_reader.cpp inside libpqhip, and libpqgen -- into lib/san/ (load with PQH_LIBDIR=lib/san and
# LD_PRELOAD of gcc's libasan + libubsan: scripts/run_sanitized.sh).  The kernels are not
# instrumented (no GPU sanitizer on this pool); they are checked against the oracle instead.
SANITIZE = os.environ.get("PQH_SANITIZE", "0") == "1" or "--sanitize" in sys.argv
SAN_FLAGS = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"]
if SANITIZE:
    LIBDIR = os.path.join(LIBDIR, "san")


def _san_link():
    gcc_dir = os.path.dirname(subprocess.check_output(["gcc", "-print-file-name=libasan.so"], text=True).strip())
    return ["-L" + gcc_dir, "-Wl,-rpath," + gcc_dir, "-lasan", "-lubsan"] if SANITIZE else []


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    deps = [os.path.join(CSRC, s) for s in sources + HEADERS] + [os.path.join(INCLUDE, "pqhip.h")]
    return any(os.path.exists(d) and os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout)
        raise RuntimeError("build failed: " + " ".join(cmd[:3]) + " ...")
    return r.stdout


def build_gen(force=False):
    out = os.path.join(LIBDIR, "libpqgen.so")
    if force or _stale(out, GEN_SRCS):
        os.makedirs(LIBDIR, exist_ok=True)
        _run(["g++", "-O2", "-g", "-std=c++17", "-shared", "-fPIC", "-Wall", "-I", INCLUDE, "-o", out]
             + (SAN_FLAGS if SANITIZE else []) + [os.path.join(CSRC, s) for s in GEN_SRCS] + ["-lz", "-lpthread"])
    return out


def source_hash():
    """sha256 (16 hex digits) of every source compiled into libpqhip.so: the build id that PMC summaries
    (profiles/*/pmc_summary.json) are stamped with, so bench.py only quotes counters of this build."""
    import hashlib

    h = hashlib.sha256()
    files = sorted(set(HOST_SRCS + HIP_SRCS + HEADERS))
    for rel in files:
        h.update(rel.encode() + b"\0")
        with open(os.path.join(CSRC, rel), "rb") as fh:
            h.update(fh.read())
    with open(os.path.join(INCLUDE, "pqhip.h"), "rb") as fh:
        h.update(b"include/pqhip.h\0" + fh.read())
    return h.hexdigest()[:16]


def _git_head():
    try:
        return subprocess.check_output(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], text=True,
                                       stderr=subprocess.DEVNULL).strip()
    except Exception:
        return None


def build_hip(force=False):
    # PQH_HIP_LIB names an experiment variant (built with its own PQH_HIPFLAGS, loaded with the same
    # variable set); the product is libpqhip.so
    out = os.path.join(LIBDIR, os.environ.get("PQH_HIP_LIB", "libpqhip.so"))
    if force or _stale(out, HOST_SRCS + HIP_SRCS):
        os.makedirs(LIBDIR, exist_ok=True)
        objs = []
        bdir = os.path.join(PKG, "build", ("san-" if SANITIZE else "") + os.path.basename(out))
        os.makedirs(bdir, exist_ok=True)
        sh = source_hash()
        for s in HIP_SRCS:
            o = os.path.join(bdir, os.path.basename(s) + ".o")
            _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
                  "-munsafe-fp-atomics", "-I", INCLUDE, f'-DPQH_SOURCE_HASH="{sh}"']
                 + os.environ.get("PQH_HIPFLAGS", "").split() + ["-c", os.path.join(CSRC, s), "-o", o])
            objs.append(o)
        for s in HOST_SRCS:
            o = os.path.join(bdir, os.path.basename(s) + ".o")
            _run(["g++", "-O2", "-g", "-std=c++17", "-fPIC", "-Wall", "-I", INCLUDE,
                  "-I", "/opt/rocm/include", "-D__HIP_PLATFORM_AMD__"] + (SAN_FLAGS if SANITIZE else [])
                 + ["-c", os.path.join(CSRC, s), "-o", o])
            objs.append(o)
        _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs + ["-lz", "-lpthread"]
             + _san_link())
        import json

        # (travels with the tree to the GPU box, which has no .git: the commit the sources were built at)
        with open(out + ".buildinfo.json", "w") as fh:
            json.dump({"source_hash": sh, "git_head": _git_head(),
                       "hipflags": os.environ.get("PQH_HIPFLAGS", "")}, fh)
    return out


def build_all(force=False):
    return build_gen(force), build_hip(force)


if __name__ == "__main__":
    for p in build_all(force="--force" in sys.argv):
        print(p)
