"""parquet-go_amd — MI355X-native Parquet column-chunk page decoder.

A drop-in for ONE hot path of github.com/fraugster/parquet-go: decoding the pages of column
chunks (the reference's pageReader.read + readValues, chunk_reader.go:182-362, page_v1.go,
page_v2.go, page_dict.go, hybrid_decoder.go, deltabp_decoder.go, type_*.go).  The decode runs as
hand-written HIP kernels for gfx950 behind the C-ABI of include/pqhip.h (libpqhip.so); this Python
package mirrors the reference's reader interface on top of that ABI (see reader.py).
"""
from . import _lib  # noqa: F401

__all__ = ["reader", "records", "assemble", "writer", "native"]


def __getattr__(name):
    import importlib

    if name in ("reader", "records", "assemble", "writer", "native", "datasets", "build", "shard"):
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
