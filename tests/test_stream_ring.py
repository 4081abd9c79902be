"""The streaming ring's bookkeeping (reader.RowGroupStream, inline and threaded) on the CPU, with
stand-ins for the native file / context / batch: every range handed out once and in order, never
more ranges open than slots, each slot used by one range at a time, everything closed after a
full pass, an abandoned pass and a failing walk or batch creation (the error reaches the caller).
The GPU run of the same ring is tests/test_gpu_stream.py."""
import threading
import time

import pytest

from conftest import load_package

pq = load_package()
native, reader = pq.native, pq.reader


class Book:
    def __init__(self, slots):
        self.lock = threading.Lock()
        self.open_hb = set()
        self.open_batches = set()
        self.slot_user = [None] * slots
        self.max_open = 0
        self.errors = []


class FakeCtx:
    def __init__(self, book, slot):
        self.book, self.slot = book, slot

    def pinned_bytes(self):
        return 0

    def close(self):
        pass


class FakeHB:
    payload_bytes = 1

    def __init__(self, book, ctx, a):
        self.book, self.ctx, self.a = book, ctx, a
        with book.lock:
            if book.slot_user[ctx.slot] is not None:
                book.errors.append(f"slot {ctx.slot} walked while range {book.slot_user[ctx.slot]} holds it")
            book.slot_user[ctx.slot] = a
            book.open_hb.add(self)
            book.max_open = max(book.max_open, len(book.open_hb))

    def close(self):
        with self.book.lock:
            if self in self.book.open_hb:
                self.book.open_hb.discard(self)
                self.book.slot_user[self.ctx.slot] = None


class FakeBatch:
    fail_at = None

    def __init__(self, ctx, hb):
        if FakeBatch.fail_at is not None and hb.a == FakeBatch.fail_at:
            raise native.PqhError(1, "staged batch failed")
        self.book, self.hb = hb.book, hb
        with self.book.lock:
            self.book.open_batches.add(self)

    @classmethod
    def staged(cls, ctx, hb):
        return cls(ctx, hb)

    def run_staged(self):
        time.sleep(0.001)

    def sync(self):
        time.sleep(0.001)

    def close(self):
        with self.book.lock:
            self.book.open_batches.discard(self)


class FakeFile:
    def __init__(self, book, nrg, fail_at=None):
        self.book, self.num_row_groups, self.fail_at = book, nrg, fail_at

    def load(self, a, b, columns, validate_crc=False, ctx=None, device_snappy=False, device_gzip=False):
        if self.fail_at is not None and a == self.fail_at:
            raise native.PqhError(2, "walk failed")
        time.sleep(0.002)
        return FakeHB(self.book, ctx, a)


@pytest.fixture
def fake(monkeypatch):
    books = []

    def make(slots):
        book = Book(slots)
        books.append(book)
        it = iter(range(slots))
        monkeypatch.setattr(native, "Context", lambda device=0, streaming=False: FakeCtx(book, next(it)))
        return book

    monkeypatch.setattr(native, "Batch", FakeBatch)
    FakeBatch.fail_at = None
    yield make
    FakeBatch.fail_at = None


def stream(book, nrg, per_range, slots, threaded, fail_walk=None):
    return reader.RowGroupStream(FakeFile(book, nrg, fail_walk), [0], per_range=per_range, slots=slots,
                                 threaded=threaded)


def assert_all_closed(book):
    assert not book.open_hb and not book.open_batches, (book.open_hb, book.open_batches)
    assert not book.errors, book.errors


@pytest.mark.parametrize("threaded", [False, True])
@pytest.mark.parametrize("slots", [1, 2, 3, 5])
def test_every_range_once_in_order(fake, threaded, slots):
    book = fake(slots)
    st = stream(book, 23, 2, slots, threaded)
    for _ in range(2):
        got = [(a, b) for a, b, batch, hb in st]
        assert got == [(a, min(a + 2, 23)) for a in range(0, 23, 2)]
        assert_all_closed(book)
    assert book.max_open <= slots
    st.close()


@pytest.mark.parametrize("threaded", [False, True])
def test_abandoned_pass_releases_every_slot(fake, threaded):
    book = fake(3)
    st = stream(book, 40, 1, 3, threaded)
    for k, (a, b, batch, hb) in enumerate(st):
        if k == 4:
            break
    assert_all_closed(book)
    assert [a for a, _, _, _ in st] == list(range(40))
    assert_all_closed(book)


@pytest.mark.parametrize("threaded", [False, True])
def test_walk_error_reaches_the_caller(fake, threaded):
    book = fake(3)
    st = stream(book, 20, 2, 3, threaded, fail_walk=10)
    seen = []
    with pytest.raises(native.PqhError, match="walk failed"):
        for a, b, batch, hb in st:
            seen.append(a)
    assert seen == [0, 2, 4, 6, 8]
    assert_all_closed(book)


@pytest.mark.parametrize("threaded", [False, True])
def test_batch_error_reaches_the_caller(fake, threaded):
    book = fake(2)
    FakeBatch.fail_at = 6
    st = stream(book, 20, 3, 2, threaded)
    seen = []
    with pytest.raises(native.PqhError, match="staged batch failed"):
        for a, b, batch, hb in st:
            seen.append(a)
    assert seen == [0, 3]
    assert_all_closed(book)
