"""Host-side mirror of the reference reader interface on top of the C-ABI.

Mirrors github.com/fraugster/parquet-go's FileReader (file_reader.go:32-351) for the decode path:
  NewFileReader(source, *columns)   -> FileReader   (NewFileReaderWithOptions + WithColumns)
  FileReader.RowGroupCount()                          (file_reader.go:242-245)
  FileReader.NumRows()                                (file_reader.go:247-250)
  FileReader.SeekToRowGroup(i) / SkipRowGroup()       (file_reader.go:187-198, 275-277)
  FileReader.PreLoad()                                (file_reader.go:280-288): the row group's
      chunks are walked on the host (thrift + codecs) and decoded on the GPU in ONE batch
  FileReader.ReadColumns()          -> {path: ColumnData}: columnar results of readValues for
      every page of the chunk (values, dLevel, rLevel) — the "throughput path" of SURVEY.md §8(b)
  FileReader.NextRow() / NextBatch(n)  (file_reader.go:258-272): records assembled columnar from
      the device's nesting outputs (assemble.py), or value by value (records.py) for the row groups
      where the reference's assembly quirks need it
Errors follow the reference: ReadColumns raises DecodeError (status, phase, index and page of the
FIRST error in decode order) for any failing chunk; the row-group cursor fails a row group only on
readChunk errors (walker, codecs, page load), and NextRow raises a readValues error at the row that
reaches the failing page (records.py).
"""
import queue
import threading
import time
from collections import deque

import numpy as np

from . import native

BOOLEAN, INT32, INT64, INT96, FLOAT, DOUBLE, BYTE_ARRAY, FIXED_LEN_BYTE_ARRAY = range(8)
_DTYPE = {INT32: np.int32, INT64: np.int64, FLOAT: np.float32, DOUBLE: np.float64, BOOLEAN: np.uint8}


class DecodeError(RuntimeError):
    def __init__(self, path, status, phase=0, index=0, page=-1):
        self.path, self.status, self.phase, self.index, self.page = path, status, phase, index, page
        super().__init__(f"{path}: {native.STATUS.get(status, status)} (phase {phase}, index {index}, page {page})")


class UnsupportedCodecError(DecodeError):
    """The chunk's codec is one this library does not decode (ZSTD, or a codec registered with
    RegisterBlockCompressor, compress.go:119-129,160,182-187).  Not a property of the data: the
    reference decodes such a chunk with its own readChunk (INTEGRATION.md's loadRowGroupGPU routes
    it there); here the chunk fails at load, before any of its pages is read."""


def decode_error(path, status, phase=0, index=0, page=-1):
    cls = UnsupportedCodecError if status == native.UNSUPPORTED_CODEC else DecodeError
    return cls(path, status, phase, index, page)


class ColumnData:
    """One decoded column chunk (dense not-null values + level bytes), host copy."""

    def __init__(self, path, column, out, page_results, ctx, nest=None, page_info=None):
        self.path = path
        self.page_info = page_info or []  # [(page_type, num_values, PageResult)] of the chunk's pages
        self.physical_type, self.type_length, self.max_def, self.max_rep = column
        self.status = out.status
        self.error_page, self.error_phase, self.error_index = out.error_page, out.error_phase, out.error_index
        self.num_values = out.num_values
        self.num_non_null = out.num_non_null
        self.value_size = out.value_size
        self.pages = page_results
        self.values = None
        self.def_levels = None
        self.rep_levels = None
        self.offsets = None
        self.data = None
        self.nesting = None
        # the reference's nil INT96 values (pqh_chunk_out.value_nil): None, or uint8 per value
        self.value_nil = None
        # readChunk errors (host walker, codecs, page load / decoder init: phase 0) fail the whole row
        # group (chunk_reader.go:394-400); otherwise the outputs of the pages before the first failing
        # one stay readable, as the reference decodes page by page (data_store.go:236-260)
        self.load_error = self._load_error(out, page_info or [])
        if out.status != native.OK and self.load_error is not None:
            return
        if out.value_size > 0:
            raw = ctx.d2h_array(out.values, out.num_non_null * out.value_size)
            if self.physical_type in _DTYPE:
                self.values = raw.view(_DTYPE[self.physical_type])
            else:
                self.values = raw.reshape(-1, out.value_size) if out.value_size else raw
        elif out.offsets:
            self.offsets = ctx.d2h_array(out.offsets, out.num_non_null + 1, np.int64)
            self.data = ctx.d2h_array(out.bytes, out.num_bytes)
        if out.value_nil and out.num_nil:
            self.value_nil = ctx.d2h_array(out.value_nil, out.num_non_null)
        if out.def_levels:
            self.def_levels = ctx.d2h_array(out.def_levels, out.num_values)
        if out.rep_levels:
            self.rep_levels = ctx.d2h_array(out.rep_levels, out.num_values)
        # nesting: [(offsets int32, validity u8) per repetition level], leaf validity u8.  Also for a
        # chunk whose pages fail in readValues: the lists before the failing page are exact (every
        # offset counts only the slots before it), which is all the record assembly reads of them
        if nest is not None and nest.num_levels:
            levels = []
            for k in range(nest.num_levels):
                lv = nest.levels[k]
                levels.append((ctx.d2h_array(lv.offsets, lv.num_lists + 1, np.int32) if lv.offsets else
                               np.zeros(1, np.int32),
                               ctx.d2h_array(lv.validity, lv.num_lists) if lv.validity else np.zeros(0, np.uint8)))
            leaf = ctx.d2h_array(nest.leaf_validity, nest.num_leaf_slots) if nest.leaf_validity else \
                np.zeros(0, np.uint8)
            self.nesting = (levels, leaf)

    @staticmethod
    def _load_error(out, page_info):
        """(status, phase, index, page) of the chunk's readChunk failure, or None."""
        if out.status == native.OK:
            return None
        if out.error_phase == native.PHASE_LOAD:
            return (out.status, out.error_phase, out.error_index, out.error_page)
        for k, (pt, n, res) in enumerate(page_info):
            if res.status != native.OK and res.phase == native.PHASE_LOAD:
                return (res.status, res.phase, res.index, k)
        return None

    def raise_for_load(self):
        """readChunk (chunk_reader.go:299-362): only page-load / walker / codec errors fail here."""
        if self.load_error is not None:
            raise decode_error(self.path, *self.load_error)
        return self

    def raise_for_status(self):
        if self.status != native.OK:
            raise decode_error(self.path, self.status, self.error_phase, self.error_index, self.error_page)
        return self

    def to_pylist(self):
        """Values as Python objects in reference order (bytes for byte arrays / FLBA / INT96)."""
        if self.values is not None:
            if self.values.ndim == 2:
                return [bytes(r) for r in self.values]
            if self.physical_type == BOOLEAN:
                return [bool(v) for v in self.values]
            return self.values.tolist()
        if self.offsets is None:
            return []
        d = self.data.tobytes()
        return [d[self.offsets[i]:self.offsets[i + 1]] for i in range(len(self.offsets) - 1)]


def batch_columns(ctx, file, batch, hb, columns):
    """ColumnData of every chunk of a synchronised batch, in (row group, column) order."""
    cols = file.columns()
    res = batch.page_results(hb.num_pages)
    pages = hb.pages()
    out = []
    for i, ch in enumerate(hb.chunks()):
        path, pt, tl, md, mr = cols[columns[i % len(columns)]]
        span = range(ch.first_page, ch.first_page + ch.num_pages)
        pr = [res[p] for p in span]
        o = batch.chunk_out(i)  # (its status orders walker, load and readValues errors as the reference)
        info = [(pages[p].page_type, pages[p].num_values, res[p]) for p in span]
        out.append(ColumnData(path, (pt, tl, md, mr), o, pr, ctx, batch.nesting(i) if mr > 0 else None, info))
    return out


def decode_chunks(ctx, file, rg_begin, rg_end, columns, validate_crc=False, return_batch=False, staged_runs=0,
                  device_snappy=False, device_gzip=False):
    """Walk (host) and decode (GPU) the chunks of `columns` in row groups [rg_begin, rg_end).

    staged_runs > 0: end-to-end mode -- the page images stay in pinned host memory and each of the
    `staged_runs` runs copies them to HBM on the copy stream ahead of the decode.
    device_snappy / device_gzip: SNAPPY / GZIP pages are decompressed on the device (k_snappy /
    k_gzip) instead of the host.
    Returns a list of ColumnData in (row group, column) order."""
    hb = file.load(rg_begin, rg_end, columns, validate_crc, device_snappy=device_snappy, device_gzip=device_gzip)
    if staged_runs:
        batch = native.Batch.staged(ctx, hb)
        for _ in range(staged_runs):
            batch.run_staged()
    else:
        batch = native.Batch.from_host(ctx, hb)
        batch.run()
    batch.sync()
    out = batch_columns(ctx, file, batch, hb, columns)
    if return_batch:
        return out, batch, hb
    batch.close()
    hb.close()
    return out


class RowGroupStream:
    """End-to-end streaming of a file's row groups through a bounded ring (SURVEY.md §8(d)
    end-to-end mode; north_star: "decompressed page buffers are staged in HBM with pinned
    hipMemcpyAsync on a side stream").  The reference reads a row group at a time --
    readRowGroupData (chunk_reader.go:375-404) walks, reads and decompresses every page of the
    selected chunks (readPageBlock / newBlockReader, chunk_reader.go:161-180, compress.go:131-152)
    before decoding -- and so does this reader, for ranges of `per_range` row groups, with `slots`
    ranges in flight:

      * slot s is a streaming context (native.CTX_STREAMING): one stream of its own (copy, zero
        fills and decode in order), its own pinned payload pool and device arena, so nothing a slot
        waits for belongs to another slot;
      * range i is walked on the host (thrift headers, CRC, decompression) straight into slot
        i % slots's pinned block, then its batch copies it to HBM on the slot's stream and
        decodes it behind the copy on the same stream (pqh_batch_run_staged): while range i decodes
        and ranges i+1.. copy, the host walks the next one;
      * a range's batch is handed to the caller once decoded and stays valid until the next
        iteration, which releases its slot (pinned block back to the slot's pool, the slot's arena
        reset) so that range i + slots can be walked into it -- by the caller between hand-outs
        (threaded=False) or, by default, by a walker and a submitter thread beside the caller.

    Pinned host memory is bounded by `slots` blocks (pinned_bytes()); device memory by the
    batches of `slots` ranges.  Iterating yields (rg_begin, rg_end, native.Batch, host batch)."""

    def __init__(self, file, columns, rg_begin=0, rg_end=None, per_range=4, slots=3, device=0, validate_crc=False,
                 threaded=True, device_snappy=False, device_gzip=False):
        self.file = file
        self.columns = list(columns)
        rg_end = file.num_row_groups if rg_end is None else rg_end
        self.ranges = [(a, min(a + per_range, rg_end)) for a in range(rg_begin, rg_end, per_range)]
        self.validate_crc = validate_crc
        self.load_kw = {"device_snappy": device_snappy, "device_gzip": device_gzip}
        self.threaded = threaded
        self.ctxs = [native.Context(device, streaming=True) for _ in range(max(1, slots))]
        self.walk_s = 0.0
        self.times = {"walk": 0.0, "create": 0.0, "run": 0.0, "sync": 0.0, "close": 0.0}

    def pinned_bytes(self):
        return sum(c.pinned_bytes() for c in self.ctxs)

    def column_data(self, batch, hb):
        """The ColumnData of a handed-out range (valid until the next iteration)."""
        return batch_columns(batch.ctx, self.file, batch, hb, self.columns)

    def _walk(self, i):
        a, b = self.ranges[i]
        t0 = time.perf_counter()
        hb = self.file.load(a, b, self.columns, self.validate_crc, ctx=self.ctxs[i % len(self.ctxs)], **self.load_kw)
        dt = time.perf_counter() - t0
        self.walk_s += dt
        self.times["walk"] += dt
        return hb

    def _stage(self, i, hb):
        t0 = time.perf_counter()
        try:
            batch = native.Batch.staged(self.ctxs[i % len(self.ctxs)], hb)
        except BaseException:
            hb.close()
            raise
        t1 = time.perf_counter()
        try:
            batch.run_staged()  # H2D on the slot's stream, then the decode (asynchronous)
        except BaseException:
            batch.close()
            hb.close()
            raise
        self.times["create"] += t1 - t0
        self.times["run"] += time.perf_counter() - t1
        return (i, batch, hb)

    def _submit(self, i):
        return self._stage(i, self._walk(i))

    def __iter__(self):
        return self._threaded() if self.threaded else self._inline()

    def _try_submit(self, i):
        try:
            return self._submit(i)
        except Exception as e:  # raised when the caller reaches range i (ranges fail in order)
            return e

    def _inline(self):
        """Walk + submit on the caller's thread, between the hand-outs."""
        inflight = deque()
        nxt = 0
        while nxt < len(self.ranges) and len(inflight) < len(self.ctxs):
            inflight.append(self._try_submit(nxt))
            nxt += 1
        try:
            while inflight:
                if isinstance(inflight[0], Exception):
                    raise inflight.popleft()
                i, batch, hb = inflight[0]  # stays listed (closed by the finally) until released
                t0 = time.perf_counter()
                batch.sync()  # the slot's own streams only
                self.times["sync"] += time.perf_counter() - t0
                a, b = self.ranges[i]
                yield a, b, batch, hb
                t0 = time.perf_counter()
                inflight.popleft()
                batch.close()
                hb.close()
                self.times["close"] += time.perf_counter() - t0
                if nxt < len(self.ranges):
                    inflight.append(self._try_submit(nxt))
                    nxt += 1
        finally:
            for item in inflight:
                if isinstance(item, tuple):
                    item[1].close()
                    item[2].close()

    def _threaded(self):
        """A two-stage producer beside the caller: a walker thread walks range i into its slot's
        pinned block as soon as the slot is released, a submitter thread creates the range's batch
        and starts its H2D + decode, and the caller waits only for decoded ranges (the native calls
        drop the GIL, so the three overlap: walk of range i+2, batch creation of range i+1, the copies
        and decodes in flight).  A slot is used by one thread at a time: the walker, then the
        submitter, then the caller until it releases the slot."""
        n, k = len(self.ranges), len(self.ctxs)
        staged, ready = queue.Queue(), queue.Queue()
        free = [threading.Semaphore(1) for _ in range(k)]
        stop = threading.Event()
        done = object()

        def walker():
            for i in range(n):
                free[i % k].acquire()
                if stop.is_set():
                    break
                try:
                    staged.put((i, self._walk(i)))
                except BaseException as e:  # handed on to the caller, which raises it
                    staged.put(e)
                    break
            staged.put(done)

        def submitter():
            while True:
                item = staged.get()
                if item is done:
                    return
                if isinstance(item, BaseException) or stop.is_set():
                    if isinstance(item, tuple):
                        item[1].close()
                    else:
                        ready.put(item)
                    continue
                try:
                    ready.put(self._stage(*item))
                except BaseException as e:
                    ready.put(e)

        threads = [threading.Thread(target=walker, name="RowGroupStream.walk", daemon=True),
                   threading.Thread(target=submitter, name="RowGroupStream.submit", daemon=True)]
        for th in threads:
            th.start()
        held = None
        try:
            for _ in range(n):
                item = ready.get()
                if isinstance(item, BaseException):
                    raise item
                held = item
                i, batch, hb = item
                t0 = time.perf_counter()
                batch.sync()  # the slot's own streams only
                self.times["sync"] += time.perf_counter() - t0
                a, b = self.ranges[i]
                yield a, b, batch, hb
                t0 = time.perf_counter()
                held = None
                batch.close()
                hb.close()
                self.times["close"] += time.perf_counter() - t0
                free[i % k].release()
        finally:
            stop.set()
            for sem in free:
                sem.release()
            for th in threads:
                th.join()
            if held is not None:
                held[1].close()
                held[2].close()
            while not ready.empty():
                item = ready.get_nowait()
                if isinstance(item, tuple):
                    item[1].close()
                    item[2].close()

    def close(self):
        for c in self.ctxs:
            c.close()
        self.ctxs = []


def records_error():
    from . import records

    return records.RecordError


class FileReader:
    """FileReader (file_reader.go:32-351) over the GPU decode.  The row-group cursor follows the
    reference: rowGroupPosition is 1-based once a group is loaded, advanceIfNeeded loads the next
    group when the current one is exhausted or skipped, io.EOF past the last group (EOFError)."""

    def __init__(self, source, *columns, device=0, validate_crc=False, ctx=None, columnar=True):
        self.file = native.File(source)
        self.ctx = ctx or native.Context(device)
        self.validate_crc = validate_crc
        allc = self.file.columns()
        self._paths = [c[0] for c in allc]
        if columns:
            sel = []
            for c in columns:
                if isinstance(c, int):
                    sel.append(c)
                else:
                    sel.extend(i for i, p in enumerate(self._paths) if p == c or p.startswith(c + "."))
            self.selected = sorted(set(sel))
        else:
            self.selected = list(range(len(allc)))
        self._schema = None
        self.row_group_position = 0  # f.rowGroupPosition
        self.current_record = 0       # f.currentRecord
        self.skip_row_group = False   # f.skipRowGroup
        self._loaded = None           # decoded chunks of row group row_group_position - 1
        self._rows = None             # assemble.ColumnarAssembler or records.RowAssembler over them
        self.columnar = columnar      # False: always the value-by-value records.RowAssembler
        self._pending = None          # NextBatch: the error of the call it stopped at
        self.assembled = {"columnar": 0, "value_by_value": 0}  # row groups per assembly path

    @classmethod
    def NewFileReader(cls, source, *columns, **kw):
        return cls(source, *columns, **kw)

    def RowGroupCount(self):
        return self.file.num_row_groups

    def NumRows(self):
        return self.file.num_rows

    def Columns(self):
        return [self._paths[i] for i in self.selected]

    def _read_row_group(self):  # readRowGroup (file_reader.go:200-207)
        if self.RowGroupCount() <= self.row_group_position:
            raise EOFError("EOF")
        self.row_group_position += 1
        rg = self.row_group_position - 1
        self._loaded = None
        self._rows = None
        self._pending = None  # a NextBatch error belongs to the row group it came from
        loaded = decode_chunks(self.ctx, self.file, rg, rg + 1, self.selected, self.validate_crc)
        # readRowGroupData (chunk_reader.go:375-404): column by column in schema order, the column
        # checks (skipChunk for the unselected ones), then readChunk; the first failure fails the group
        by_col = dict(zip(self.selected, loaded))
        for ci, path in enumerate(self._paths):
            st = self.file.chunk_check(rg, ci, ci in by_col)
            if st != native.OK:
                raise DecodeError(path, st, native.PHASE_LOAD, 0, -1)
            if ci in by_col:
                by_col[ci].raise_for_load()
        self._loaded = loaded

    def _advance_if_needed(self):  # advanceIfNeeded (file_reader.go:226-238)
        if (self.row_group_position == 0 or self.skip_row_group
                or self.current_record >= self.file.row_group_num_rows(self.row_group_position - 1)):
            try:
                self._read_row_group()
            except Exception:  # io.EOF or a readRowGroup error: the next call moves on (file_reader.go:228-232)
                self.skip_row_group = True
                raise
            self.current_record = 0
            self.skip_row_group = False

    def SeekToRowGroup(self, position):
        """file_reader.go:186-198: rowGroupPosition = position - 1, then readRowGroup, which loads
        RowGroups[position - 1] -- so, as in the reference, position 1 is the first row group and
        position 0 fails (the reference's index -1 panic, recovered into an error)."""
        if position < 1:
            raise IndexError(f"index out of range [{position - 1}]")
        self.row_group_position = position - 1
        self.current_record = 0
        self._pending = None
        self._read_row_group()

    def SkipRowGroup(self):
        self.skip_row_group = True
        self._pending = None

    def PreLoad(self):
        self._advance_if_needed()
        return self

    def RowGroupNumRows(self):
        self._advance_if_needed()
        return self.file.row_group_num_rows(self.row_group_position - 1)

    def ReadColumns(self):
        """The columnar throughput path: {path: ColumnData} of the current row group."""
        self.PreLoad()
        return {c.path: c.raise_for_status() for c in self._loaded}

    def _assembler(self, arrow=False):
        """The current row group's record assembly: columnar over the device's nesting outputs
        (assemble.ColumnarAssembler), else value by value (records.RowAssembler) when the row group
        breaks one of its preconditions (the reference's page-local cursors / getFirstRDLevel
        quirks)."""
        from . import assemble

        if self._schema is None:
            self._schema = self.file.schema()
        nrows = self.file.row_group_num_rows(self.row_group_position - 1)
        if self.columnar:
            leaves = {}
            for ci, c in zip(self.selected, self._loaded):
                pages = [(res.level_offset, res.status, res.phase, res.index)
                         for pt, n, res in c.page_info if pt != 2]
                levels, leaf = c.nesting if c.nesting is not None else (None, None)
                if (c.max_rep and c.nesting is None) or c.value_nil is not None:
                    break  # (Go nil values, type_int96.go:21-42: the value-by-value assembly)
                leaves[ci] = assemble.Leaf(c.path, c.max_def, c.max_rep, self.file.rep_def(ci), c.def_levels,
                                           c.rep_levels, levels, leaf,
                                           lambda c=c: assemble.dense_values(c, c.physical_type), pages, c.num_values,
                                           arrow=lambda c=c: assemble.arrow_dense(c, c.physical_type))
            else:
                try:
                    a = assemble.ColumnarAssembler(self._schema, leaves, nrows)
                    if arrow:
                        return ("arrow", a)
                    rows, errs = a.rows(), a.errors()
                    self.assembled["columnar"] += 1
                    return ("columnar", rows, errs)
                except assemble.NotColumnar:
                    pass
        return self._value_by_value()

    def _value_by_value(self):
        """records.RowAssembler over the current row group: readValues errors surface page by page,
        when the assembly reaches the failing page (ColumnStore.get -> readNextPage,
        data_store.go:236-269); rows before it are returned."""
        from . import records

        if self._schema is None:
            self._schema = self.file.schema()
        nrows = self.file.row_group_num_rows(self.row_group_position - 1)
        cols = {self.selected[i]: (c, c.physical_type, c.path) for i, c in enumerate(self._loaded)}
        self.assembled["value_by_value"] += 1
        return ("value_by_value", records.RowAssembler(self._schema, cols, nrows))

    def NextRow(self):
        """NextRow (file_reader.go:258-272): the next record as a dict, loading the next row group
        when needed; EOFError after the last row.  A readValues error surfaces at the row that
        reaches the failing page (records.RecordError), as in the reference."""
        from . import records

        if self._pending is not None:
            e, self._pending = self._pending, None
            raise e
        self._advance_if_needed()
        if self._rows is None:
            self._rows = self._assembler()
        k = self.current_record
        self.current_record += 1
        if self._rows[0] == "value_by_value":
            return self._rows[1].next_row()
        _, rows, errs = self._rows
        if k < len(rows):
            return rows[k]
        e = errs[k - len(rows)]
        # the same message and attributes as the value-by-value path (records.LeafStore._read_next_page)
        raise records.RecordError(f"{e[4]}: page {e[5]} failed to decode (status {e[1]}, phase {e[2]}, index {e[3]})",
                                  e[1], e[2], e[3], e[5])

    def NextBatch(self, n):
        """Up to n records of the current row group (the next one when it is exhausted), stopping
        before a row that fails -- that row's error is raised by the next NextRow / NextBatch call,
        exactly as the same sequence of NextRow calls would; [] at the end of the file."""
        if self._pending is not None:
            e, self._pending = self._pending, None
            raise e
        out = []
        if n <= 0:
            return out
        try:
            out.append(self.NextRow())
        except EOFError:
            return out
        nrows = self.file.row_group_num_rows(self.row_group_position - 1)
        if self._rows[0] == "columnar":  # the rest of the row group's ready rows at once
            rows = self._rows[1]
            k = self.current_record
            take = rows[k:k + n - 1]
            self.current_record += len(take)
            out.extend(take)
            return out
        while len(out) < n and self.current_record < nrows:
            try:
                out.append(self.NextRow())
            except records_error() as e:
                self._pending = e
                break
        return out

    def ReadRowGroupArrow(self):
        """The records of the current row group from the cursor on (the next row group when it is
        exhausted; None at the end of the file) as a pyarrow Table, built from the device's columnar
        outputs (assemble.ColumnarAssembler.arrow: list offsets, presence, leaf validity and the dense
        values, with no per-row Python object); assemble.drop_absent(row) of its to_pylist() rows
        equals what NextRow returns.  Rows stop before a row whose page fails to decode; that row's
        error is raised by the next NextRow / NextBatch / ReadRowGroupArrow call, as with NextBatch.
        Row groups the columnar assembly cannot describe (records.py's corner cases, nil INT96
        values) go through NextBatch's records into the table."""
        import pyarrow as pa

        from . import assemble

        if self._pending is not None:
            e, self._pending = self._pending, None
            raise e
        try:
            self._advance_if_needed()
        except EOFError:
            return None
        nrows = self.file.row_group_num_rows(self.row_group_position - 1)
        k = self.current_record
        if self._rows is None and k == 0:
            a = self._assembler(arrow=True)
            if a[0] == "arrow":
                asm = a[1]
                try:
                    # (runs the assembler's lazy checks -- leaves that disagree, instance counts,
                    # repeated leaves -- that rows() runs too: a row group that breaks one goes value
                    # by value, as NextRow does)
                    t = asm.arrow()
                except assemble.NotColumnar:
                    a = self._value_by_value()
                else:
                    self.assembled["arrow"] = self.assembled.get("arrow", 0) + 1
                    # the cursor after the table's rows: a failing row's error comes from the next call
                    # (NextRow's columnar path raises errs[k - ok_rows] there)
                    self._rows = ("columnar", [None] * asm.ok_rows, asm.errors())
                    self.current_record = asm.ok_rows
                    return t
            self._rows = a
        rows = self.NextBatch(nrows - k)
        return assemble.records_table(rows) if rows else pa.table({})

    def close(self):
        self.file.close()
