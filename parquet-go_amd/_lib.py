"""ctypes loading of the in-tree native libraries (parquet-go_amd/lib/*.so).

The product library libpqhip.so MUST be the in-tree HIP build: there is no CPU fallback.  If it
is missing, build it with `python parquet-go_amd/build.py` (or __graft_entry__.build()).
"""
import ctypes
import os

PKG = os.path.dirname(os.path.abspath(__file__))
# PQH_LIBDIR: another build of the same libraries (the sanitizer variants in lib/san)
LIBDIR = os.environ.get("PQH_LIBDIR") or os.path.join(PKG, "lib")

_gen = None
_hip = None


class NativeLibraryMissing(RuntimeError):
    pass


def _load(name, builder):
    path = os.path.join(LIBDIR, name)
    if not os.path.exists(path):
        if os.environ.get("PQH_AUTOBUILD", "1") == "1":
            from . import build as _b

            getattr(_b, builder)()
        if not os.path.exists(path):
            raise NativeLibraryMissing(f"{path} not built (python parquet-go_amd/build.py)")
    return ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


def gen():
    global _gen
    if _gen is None:
        L = _load("libpqgen.so", "build_gen")
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
        L.pqg_write.argtypes = [vp, i32, vp, i32, vp, i32, vp, vp, vp, ctypes.c_char_p, i32]
        L.pqg_write.restype = ctypes.c_int
        L.pqg_free.argtypes = [vp]
        L.pqg_hybrid_encode.argtypes = [i32, vp, i64, vp, i64]
        L.pqg_hybrid_encode.restype = i64
        L.pqg_delta_encode32.argtypes = [vp, i64, vp, i64]
        L.pqg_delta_encode32.restype = i64
        L.pqg_delta_encode64.argtypes = [vp, i64, vp, i64]
        L.pqg_delta_encode64.restype = i64
        L.pqg_stream_open.argtypes = [vp, i32, vp, ctypes.c_char_p, i32]
        L.pqg_stream_open.restype = vp
        L.pqg_stream_write.argtypes = [vp, vp, i32, vp, i32, vp, i64, vp, ctypes.c_char_p, i32]
        L.pqg_stream_write.restype = ctypes.c_int
        L.pqg_stream_finish.argtypes = [vp, vp, i64, vp, ctypes.c_char_p, i32]
        L.pqg_stream_finish.restype = ctypes.c_int
        L.pqg_stream_close.argtypes = [vp]
        L.pqg_mixed_dicts.argtypes = [ctypes.c_uint64, vp, vp]
        L.pqg_mixed_row_group.argtypes = [ctypes.c_uint64, i32, i64, vp, vp, vp, vp, vp, vp, vp, vp, i32]
        L.pqg_mixed_row_group.restype = i64
        _gen = L
    return _gen


def hip():
    global _hip
    if _hip is None:
        from . import native

        _hip = native.bind(_load(os.environ.get("PQH_HIP_LIB", "libpqhip.so"), "build_hip"))
    return _hip


def hip_path():
    return os.path.join(LIBDIR, os.environ.get("PQH_HIP_LIB", "libpqhip.so"))
