"""Extract the corrupt / foreign-writer Parquet files the reference's tests embed as Go string
literals, as binary fixtures.

Reads the reference's test files as TEXT (no Go toolchain is involved) and decodes the byte-string
literals by Go's rules for interpreted string literals (\\xhh, \\ooo, \\uhhhh, \\Uhhhhhhhh as UTF-8,
\\a \\b \\f \\n \\r \\t \\v \\\\ \\", other characters as their UTF-8 bytes; "..." + "..." concatenated):
  fuzz_test.go:11-47            TestFuzzThriftReadCrashes (6 crashers)
  type_dict_test.go:33-177      TestFuzzCrashDictDecoderDecodeValues (a parquet-cpp 1.5.1 file)
  packed_array_test.go:61       (the same parquet-cpp file, a second test)
  deltabp_decoder_test.go:5-150, 152-297   parquet-mr 1.8.0 impala ComplexTypesTbl (DELTA pages)
  chunk_reader_test.go:5-22     TestFuzzCrashReadRowGroup
  page_v1_test.go:5             TestDataPageReaderV1InitCrash
  type_bytearray_test.go:14-36  TestFuzzCrashByteArrayPlainDecoderNext
  schema_test.go:162, 241       TestFuzzCrashReadGroupSchema2 / TestFuzzCrashReadGroupSchema
Writes tests/golden/fuzz/<test name>[_<k>].bin (the file bytes, data only) and manifest.json
(name, source file:line, length, sha256).  The reference's tests assert only that reading these
files does not crash (readAllData, schema_test.go:388-403).

Run once in the build container:  python tests/golden/make_fuzz_fixtures.py
"""
import hashlib
import json
import os
import re
import sys

REF = os.environ.get("PQ_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "fuzz")
FILES = ["fuzz_test.go", "type_dict_test.go", "packed_array_test.go", "deltabp_decoder_test.go",
         "chunk_reader_test.go", "page_v1_test.go", "type_bytearray_test.go", "schema_test.go"]

_SIMPLE = {"a": 7, "b": 8, "f": 12, "n": 10, "r": 13, "t": 9, "v": 11, "\\": 92, '"': 34, "'": 39}


def go_string(lit):
    """Bytes of one Go interpreted string literal body (between the quotes)."""
    out = bytearray()
    i = 0
    while i < len(lit):
        c = lit[i]
        if c != "\\":
            out += c.encode("utf-8")
            i += 1
            continue
        e = lit[i + 1]
        if e in _SIMPLE:
            out.append(_SIMPLE[e])
            i += 2
        elif e == "x":
            out.append(int(lit[i + 2:i + 4], 16))
            i += 4
        elif e in "01234567":
            out.append(int(lit[i + 1:i + 4], 8))
            i += 4
        elif e == "u":
            out += chr(int(lit[i + 2:i + 6], 16)).encode("utf-8")
            i += 6
        elif e == "U":
            out += chr(int(lit[i + 2:i + 10], 16)).encode("utf-8")
            i += 10
        else:
            raise ValueError(f"unknown escape \\{e}")
    return bytes(out)


_LIT = re.compile(r'"((?:[^"\\\n]|\\.)*)"')


def literal_chain(text, pos):
    """The concatenation "a" + "b" + ... starting at the first quote at/after pos."""
    parts = []
    while True:
        m = _LIT.match(text, pos)
        if not m:
            raise ValueError(f"no string literal at {pos}")
        parts.append(go_string(m.group(1)))
        pos = m.end()
        rest = re.match(r"\s*\+\s*", text[pos:])
        if not rest:
            return b"".join(parts), pos
        pos += rest.end()


def extract(name):
    text = open(os.path.join(REF, name)).read()
    out = []
    for m in re.finditer(r"func (Test\w+)\(", text):
        test = m.group(1)
        end = text.find("\nfunc ", m.end())
        body_end = len(text) if end < 0 else end
        k = 0
        pos = m.end()
        while True:
            q = text.find('"PAR1', pos, body_end)
            if q < 0:
                break
            data, pos = literal_chain(text, q)
            line = text.count("\n", 0, q) + 1
            out.append((f"{test}_{k}" if k or text.find('"PAR1', pos, body_end) >= 0 else test, f"{name}:{line}", data))
            k += 1
    return out


def main():
    if not os.path.isdir(REF):
        sys.exit(f"reference {REF} not found")
    os.makedirs(OUT, exist_ok=True)
    manifest = []
    for name in FILES:
        for test, src, data in extract(name):
            fn = f"{test}.bin"
            with open(os.path.join(OUT, fn), "wb") as f:
                f.write(data)
            manifest.append({"file": fn, "test": test, "source": src, "length": len(data),
                             "sha256": hashlib.sha256(data).hexdigest()})
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump({"reference_tests_assert": "no panic (readAllData, schema_test.go:388-403)",
                   "fixtures": manifest}, f, indent=1)
    for m in manifest:
        print(f"{m['file']:60s} {m['length']:6d} B  {m['source']}")


if __name__ == "__main__":
    main()
