"""The codec boundary (reference compress.go:16-33,119-187): the reference decodes
a chunk with whatever its compressors registry holds -- UNCOMPRESSED, GZIP, SNAPPY and ZSTD after
init (:182-187), plus codecs a program adds with RegisterBlockCompressor (:160) -- and fails a codec
it has no compressor for with "decompression failed: method %q is not supported" at the chunk's first
page block.  libpqhip decodes UNCOMPRESSED / SNAPPY / GZIP.  A chunk whose codec the caller's
registry holds but the library does not decode must not look like a corrupt page: the walker stops
it before reading any page with PQH_ERR_UNSUPPORTED_CODEC (the shim then calls the reference's own
readChunk); an unregistered codec fails exactly as the reference fails it.

Files written here by pyarrow 25 with per-column codecs; the oracle restates the reference's walk
with the same registry (ZSTD decoded through pyarrow's codec: the format defines the bytes)."""
import io

import numpy as np
import pytest

from oracle import oracle as O

UNSUPPORTED_CODEC = 35
DECOMPRESS = 23


def _file(version="1.0", page_v2=False, n=6000, seed=1):
    import pyarrow as pa
    import pyarrow.parquet as pqa

    rng = np.random.default_rng(seed)
    t = pa.table({"z": pa.array(rng.integers(-99, 99, n)),
                  "s": pa.array([str(x) for x in rng.integers(0, 1000, n)]),
                  "u": pa.array(rng.random(n)),
                  "g": pa.array(rng.integers(0, 5, n).astype(np.int32)),
                  "l": pa.array(rng.integers(0, 9, n).astype(np.int32)),
                  "z2": pa.array([None if x % 7 == 0 else f"k{x}" for x in rng.integers(0, 300, n)])})
    buf = io.BytesIO()
    pqa.write_table(t, buf, compression={"z": "zstd", "s": "snappy", "u": "none", "g": "gzip", "l": "lz4",
                                         "z2": "zstd"},
                    row_group_size=2500, data_page_size=4096, data_page_version="2.0" if page_v2 else "1.0")
    return buf.getvalue()


def _codecs(fr):
    return [c[3][4] for c in fr.row_groups[0][1]]


@pytest.mark.parametrize("v2", [False, True])
def test_walk_reports_registered_codecs(pq, v2):
    """Default registry: the ZSTD chunks fail at load with UNSUPPORTED_CODEC and no page listed (the
    oracle -- the reference -- decodes them); the LZ4 chunk (in no registry) fails as the reference
    fails it; every other chunk is walked exactly as the oracle walks it."""
    data = _file(page_v2=v2)
    fr = O.FileReader(data)
    codecs = _codecs(fr)
    assert O.ZSTD in codecs and 1 in codecs and 2 in codecs and 0 in codecs
    lz4 = [c for c in codecs if c not in (0, 1, 2, O.ZSTD)]
    assert lz4, codecs  # (pyarrow's 'lz4' codec id: LZ4_RAW)
    f = pq.native.File(data)
    ncols = len(f.columns())
    hb = f.load(0, f.num_row_groups, list(range(ncols)))
    seen = set()
    for k, ch in enumerate(hb.chunks()):
        rg, ci = divmod(k, ncols)
        och = fr.read_chunk(rg, ci)
        codec = codecs[ci]
        if codec == O.ZSTD:
            assert ch.host_status == UNSUPPORTED_CODEC and ch.num_pages == 0
            # the reference reads it (V1); pyarrow's V2 pages may store a values section
            # uncompressed (is_compressed = false), which the reference decompresses regardless
            # (page_v2.go:125) and fails on -- its outcome, which the shim's routing reproduces
            assert (och.status == 0 and och.pages) or (v2 and och.status == DECOMPRESS)
            seen.add("zstd")
        elif codec in lz4:
            assert ch.host_status == och.status == DECOMPRESS  # "method ... is not supported"
            seen.add("unregistered")
        else:
            assert ch.host_status == och.status and (v2 or och.status == 0)
            if och.status == 0:
                assert ch.num_pages == len(och.pages) + (och.dict_page is not None)
    assert seen == {"zstd", "unregistered"}
    hb.close()
    f.close()


def test_registry_follows_the_caller(pq):
    """pqh_file_set_codecs = the caller's registry: without ZSTD the ZSTD chunks fail as the
    reference without a ZSTD compressor fails them (DECOMPRESS, like the oracle with the same
    registry); with LZ4_RAW registered (RegisterBlockCompressor) the LZ4 chunk becomes
    UNSUPPORTED_CODEC too."""
    data = _file()
    base = O.FileReader(data)
    codecs = _codecs(base)
    lz4 = next(c for c in codecs if c not in (0, 1, 2, O.ZSTD))
    # (the reference's init registers UNCOMPRESSED / GZIP / SNAPPY and nothing unregisters a codec, so
    # every registry holds them; the library always decodes them)
    for reg in ([0, 1, 2], [0, 1, 2, O.ZSTD, lz4], [0, 1, 2, lz4]):
        fr = O.FileReader(data, codecs=reg)
        f = pq.native.File(data)
        f.set_codecs(reg)
        ncols = len(f.columns())
        hb = f.load(0, f.num_row_groups, list(range(ncols)))
        for k, ch in enumerate(hb.chunks()):
            rg, ci = divmod(k, ncols)
            och = fr.read_chunk(rg, ci)
            if codecs[ci] in reg and codecs[ci] not in (0, 1, 2):
                assert ch.host_status == UNSUPPORTED_CODEC and ch.num_pages == 0, (reg, ci)
            else:
                assert ch.host_status == och.status, (reg, ci, ch.host_status, och.status)
        hb.close()
        f.close()


@pytest.mark.gpu
@pytest.mark.parametrize("v2", [False, True])
def test_decode_around_unsupported_codecs(pq, v2):
    """GPU: the ZSTD chunks report UNSUPPORTED_CODEC (reader.UnsupportedCodecError), never
    DECOMPRESS; every other chunk of the same batch decodes bit for bit as the oracle decodes it; a
    FileReader over the other columns reads every row group."""
    from test_gpu_parity import assert_chunk, oracle_chunk

    data = _file(page_v2=v2)
    fr = O.FileReader(data)
    codecs = _codecs(fr)
    ctx = pq.native.Context(0)
    f = pq.native.File(data)
    ncols = len(f.columns())
    got = pq.reader.decode_chunks(ctx, f, 0, f.num_row_groups, list(range(ncols)))
    for k, col in enumerate(got):
        rg, ci = divmod(k, ncols)
        if codecs[ci] == O.ZSTD:
            assert col.status == UNSUPPORTED_CODEC
            with pytest.raises(pq.reader.UnsupportedCodecError):
                col.raise_for_status()
        else:
            assert_chunk(col, oracle_chunk(fr, rg, ci), where=f"rg{rg} col{ci}")
    if v2:  # (pyarrow's uncompressed V2 value sections fail the reference's SNAPPY / GZIP read)
        f.close()
        return
    others = [ci for ci, c in enumerate(codecs) if c in (0, 1, 2)]
    r = pq.reader.FileReader(data, *others, ctx=ctx)
    for _ in range(r.RowGroupCount()):
        cols = r.ReadColumns()
        assert len(cols) == len(others)
        r.SkipRowGroup()
    r.close()
    f.close()
