"""The reference's page walk with a pluggable data-page reader (test infrastructure).

`read_pages` restates readChunk + readPages (reference chunk_reader.go:299-362, :182-263) over an
`OffsetReader` (helpers.go:39-64): the loop reads a thrift PageHeader from the SAME reader the page
readers read their blocks from, until TotalCompressedSize - r.Count() <= 0.  A page reader that
consumes the wrong number of bytes therefore desynchronises the walk exactly as it would in Go.

Two data-page readers plug into it:
  * `OraclePage`  — dataPageReaderV1/V2 (page_v1.go:87-122, page_v2.go:79-131) over the oracle:
                    readPageBlock + newBlockReader + decoders, readValues from oracle.decode_page;
  * `ShimPage`    — INTEGRATION.md's gpuPageReader: `read` consumes CompressedPageSize bytes from
                    r (io.CopyN after readPageBlock's size check) and reports the batch's load
                    error for its page; `readValues(size)` is one pqh_batch_page_read of the
                    batch page `index` = chunk.first_page + (dictionary page ? 1 : 0) + the data
                    page's ordinal.  `backend` supplies readValues: "device" = Batch.page_read (GPU),
                    "host" = the host batch's page image decoded by the oracle (CPU: pins the page
                    index mapping and the byte accounting without a GPU).
The dictionary page stays with the reference's own dictPageReader (page_dict.go:35-72), as in the
shim.
"""
import numpy as np

from oracle import oracle as O


class WalkError(Exception):
    def __init__(self, status, page, phase=O.PHASE_LOAD, index=0):
        super().__init__(f"status {status} at data page {page}")
        self.status, self.page, self.phase, self.index = status, page, phase, index


class OffsetReader:
    """helpers.go:39-64: Read advances offset and count; Seek moves both (count by the distance)."""

    def __init__(self, data, offset):
        self.data, self.offset, self.count = data, offset, 0

    def read(self, n):  # io.ReadAll(io.LimitReader(r, n)): whatever is there, no error when short
        b = self.data[self.offset:self.offset + max(0, n)]
        self.offset += len(b)
        self.count += len(b)
        return b

    def seek(self, pos):
        self.count += pos - self.offset
        self.offset = pos

    def read_thrift(self):  # readThrift (helpers.go:103-109) on the stream
        rd = O.CompactReader(self.data, min(self.offset, len(self.data)))
        ph = rd.read("PageHeader")
        n = rd.pos - min(self.offset, len(self.data))
        self.offset += n
        self.count += n
        return ph


def _inflate(codec, blk, csz, usz):  # newBlockReader (compress.go:131-152)
    if csz < 0 or usz < 0:
        return None, O.ERR_PAGE_HEADER
    if len(blk) != csz:
        return None, O.ERR_DECOMPRESS
    try:
        img = O.decompress(codec, blk, usz)
    except Exception:
        return None, O.ERR_DECOMPRESS
    return (img, O.OK) if len(img) == usz else (None, O.ERR_DECOMPRESS)


class OraclePage:
    """dataPageReaderV1 / V2 over the oracle."""

    def __init__(self, desc, dictionary):
        self.desc, self.dictionary = desc, dictionary
        self.res = None
        self.pos = 0

    def read(self, r, ph, codec, validate_crc):
        usize, csize = ph[2], ph[3]
        if ph[1] == O.DATA_PAGE:
            h = ph.get(5)
            if h is None or h[1] < 0:
                return O.ERR_PAGE_HEADER
            if csize < 0 or usize < 0:
                return O.ERR_PAGE_HEADER
            blk = r.read(csize)
            if validate_crc and 4 in ph and (O.zlib.crc32(blk) & 0xFFFFFFFF) != (ph[4] & 0xFFFFFFFF):
                return O.ERR_CRC
            img, st = _inflate(codec, blk, csize, usize)
            if st:
                return st
            page = (O.DATA_PAGE, h[1], h[2], 0, 0, img)
        else:
            h = ph.get(8)
            if h is None or h[1] < 0 or h[5] < 0 or h[6] < 0:
                return O.ERR_PAGE_HEADER
            if O.select(self.desc, h[4]) != O.OK:
                return O.ERR_UNSUPPORTED
            if csize < 0 or usize < 0:
                return O.ERR_PAGE_HEADER
            blk = r.read(csize)
            if validate_crc and 4 in ph and (O.zlib.crc32(blk) & 0xFFFFFFFF) != (ph[4] & 0xFFFFFFFF):
                return O.ERR_CRC
            dl, rl = h[5], h[6]
            if rl + dl > len(blk):
                return O.ERR_PAGE_HEADER
            vals, st = _inflate(codec, blk[rl + dl:], csize - rl - dl, usize - rl - dl)
            if st:
                return st
            page = (O.DATA_PAGE_V2, h[1], h[4], dl, rl, blk[:rl + dl] + vals)
        self.res = O.decode_page(self.desc, *page, self.dictionary)
        if self.res.status and self.res.phase == O.PHASE_LOAD:
            return self.res.status
        return O.OK

    def num_values(self):
        return self.res.num_values

    def read_values(self, size):
        return slice_result(self.res, self.pos, size, self)


def boxed_with_nil(raw, size, mask):
    """Fixed-width values as the list boxValues builds when some are the reference's nil (a short
    INT96 value, type_int96.go:21-42): bytes per value, None for a nil one."""
    return [None if mask[i] else bytes(raw[i * size:(i + 1) * size]) for i in range(len(mask))]


def slice_result(res, first, size, reader):
    """readValues(size) from a whole-page oracle result: (status, phase, index, values, def, rep).
    Mirrors pqh_batch_page_read's contract (include/pqhip.h): a level error fails every call of the
    page, a value error fails the call whose values reach it (partial counts are not returned)."""
    n = res.num_values
    s0, s1 = min(first, n), min(n, first + size)
    reader.pos = s1
    if res.status and res.phase != O.PHASE_VALUES:
        return res.status, res.phase, None, None, None
    d = res.def_levels[s0:s1] if res.def_levels is not None else None
    rl = res.rep_levels[s0:s1] if res.rep_levels is not None else None
    nn0 = int(np.count_nonzero(res.def_levels[:s0] == reader.desc[2])) if res.def_levels is not None else s0
    nn1 = int(np.count_nonzero(d == reader.desc[2])) if d is not None else s1 - s0
    if res.status and res.index < nn0 + nn1:
        return res.status, res.phase, None, None, None
    if res.offsets is not None:
        offs = res.offsets[nn0:nn0 + nn1 + 1]
        vals = (offs - offs[0], res.values[offs[0]:offs[-1]])
    else:
        vs = res.value_size
        vals = res.values[nn0 * vs:(nn0 + nn1) * vs]
        if res.nil is not None and res.nil[nn0:nn0 + nn1].any():
            vals = boxed_with_nil(vals, vs, res.nil[nn0:nn0 + nn1])
    return O.OK, 0, vals, d, rl


class ShimPage:
    """INTEGRATION.md gpuPageReader over one chunk of a host batch (and its decoded batch)."""

    def __init__(self, shim, ordinal):
        self.shim, self.ordinal = shim, ordinal
        c = shim.chunk
        self.index = c.first_page + shim.has_dict + ordinal  # batch page index of the data page
        self.pos = 0
        self.desc = shim.desc

    def read(self, r, ph, codec, validate_crc):
        csize, usize = ph[3], ph[2]
        if csize < 0 or usize < 0:  # readPageBlock's size check before the read (chunk_reader.go:162-164)
            return O.ERR_PAGE_HEADER
        r.read(csize)  # io.CopyN(io.Discard, r, CompressedPageSize): the bytes readPageBlock consumes
        return self.shim.load_error(self.ordinal)

    def num_values(self):
        return self.shim.pages[self.index].num_values

    def read_values(self, size):
        return self.shim.read_values(self, size)


class Shim:
    """The shim's view of one chunk of a batch: the host batch's chunk table (pqh_host_batch_chunks /
    pages), plus readValues from the device batch or, on the CPU, from the host images."""

    def __init__(self, hb, chunk_index, desc, backend="host", batch=None):
        self.hb, self.k, self.desc, self.backend, self.batch = hb, chunk_index, desc, backend, batch
        self.chunk = hb.chunks()[chunk_index]
        self.pages = hb.pages()
        self.payload = hb.payload()
        c = self.chunk
        self.has_dict = int(c.num_pages > 0 and self.pages[c.first_page].page_type == O.DICTIONARY_PAGE)
        self.listed = c.num_pages - self.has_dict  # data pages the host walk read
        self._dict = None
        self._res = {}
        if backend == "device":
            self.out = batch.chunk_out(chunk_index)

    def dictionary(self):
        if self.has_dict and self._dict is None:
            p = self.pages[self.chunk.first_page]
            img = self.payload[p.image_offset:p.image_offset + p.image_len].tobytes()
            self._dict = O.decode_dict_page(self.desc, p.num_values, p.encoding, img)
        return self._dict

    def _page_result(self, index):
        if index not in self._res:
            p = self.pages[index]
            img = self.payload[p.image_offset:p.image_offset + p.image_len].tobytes()
            self._res[index] = O.decode_page(self.desc, p.page_type, p.num_values, p.encoding,
                                             p.def_levels_byte_length, p.rep_levels_byte_length, img, self.dictionary())
        return self._res[index]

    def load_error(self, ordinal):
        """The status `read` returns for data page `ordinal`: the batch's readChunk error when it
        belongs to this page, else OK."""
        if ordinal >= self.listed:  # the host walk stopped at this page
            return self.chunk.host_status
        index = self.chunk.first_page + self.has_dict + ordinal
        if self.backend == "device":
            o = self.out
            if o.status and o.error_phase == O.PHASE_LOAD and o.error_page == index:
                return o.status
            return O.OK
        r = self._page_result(index)
        return r.status if r.status and r.phase == O.PHASE_LOAD else O.OK

    def read_values(self, page, size):
        if self.backend == "device":
            nil = []
            pv, vals, d, rl = self.batch.page_read(page.index, page.pos, size, nil=nil)
            page.pos += pv.num_slots
            if pv.status:
                return pv.status, pv.phase, None, None, None
            c = self.desc
            if pv.num_nil:  # boxValues with its nil slots (INTEGRATION.md readValues): one entry per value
                vals = boxed_with_nil(vals.tobytes(), pv.value_size, nil[0])
            return O.OK, 0, (vals if pv.value_size > 0 else (vals[0], vals[1].tobytes())), \
                (d if c[2] > 0 else None), (rl if c[3] > 0 else None)
        return slice_result(self._page_result(page.index), page.pos, size, page)


def read_pages(data, fr, rg, ci, make_page, validate_crc=False, dict_for=None):
    """readChunk + readPages (chunk_reader.go:299-362, :182-263).  make_page(ordinal, dictionary) ->
    a data-page reader.  Returns (pages, dictionary, error or None)."""
    st = fr.chunk_check(rg, ci)
    if st:
        return [], None, WalkError(st, 0)
    md = fr.row_groups[rg][1][ci][3]
    desc = fr.columns[ci].desc()
    r = OffsetReader(fr.data, md.get(11, md[9]))
    total, codec = md[7], md[4]
    pages, dictionary = [], None
    while total - r.count > 0:
        try:
            ph = r.read_thrift()
        except O.ThriftError:
            return pages, dictionary, WalkError(O.ERR_THRIFT, len(pages))
        if ph[1] == O.DICTIONARY_PAGE:  # the reference's dictPageReader (kept by the shim)
            if dictionary is not None:
                return pages, dictionary, WalkError(O.ERR_DICT_PAGE, len(pages))
            if desc[0] == O.BOOLEAN:
                return pages, dictionary, WalkError(O.ERR_UNSUPPORTED, len(pages))
            dh = ph.get(7)
            if dh is None or dh[1] < 0:
                return pages, dictionary, WalkError(O.ERR_PAGE_HEADER, len(pages))
            if dh[2] not in (0, 2):
                return pages, dictionary, WalkError(O.ERR_DICT_PAGE, len(pages))
            if ph[3] < 0 or ph[2] < 0:
                return pages, dictionary, WalkError(O.ERR_PAGE_HEADER, len(pages))
            blk = r.read(ph[3])
            if validate_crc and 4 in ph and (O.zlib.crc32(blk) & 0xFFFFFFFF) != (ph[4] & 0xFFFFFFFF):
                return pages, dictionary, WalkError(O.ERR_CRC, len(pages))
            img, st = _inflate(codec, blk, ph[3], ph[2])
            if st:
                return pages, dictionary, WalkError(st, len(pages))
            dictionary = O.decode_dict_page(desc, dh[1], dh[2], img)
            if dictionary.status:
                return pages, dictionary, WalkError(dictionary.status, len(pages))
            if 11 in md and md[11] != r.offset:  # back to DataPageOffset
                r.seek(md[9])
            continue
        if ph[1] not in (O.DATA_PAGE, O.DATA_PAGE_V2):
            return pages, dictionary, WalkError(O.ERR_PAGE_HEADER, len(pages))
        if ph[1] == O.DATA_PAGE:  # init: the level decoders' encodings (page_v1.go:65-85)
            h = ph.get(5)
            if h is not None:
                c = fr.columns[ci]
                if (c.max_rep > 0 and h[4] != 3) or (c.max_def > 0 and h[3] != 3):
                    return pages, dictionary, WalkError(O.ERR_UNSUPPORTED, len(pages))
        p = make_page(len(pages), dictionary)
        st = p.read(r, ph, codec, validate_crc)
        if st:
            return pages, dictionary, WalkError(st, len(pages))
        pages.append(p)
    return pages, dictionary, None
