"""Extract the reference's bit-packing known-answer tables into JSON fixtures.

Reads the test tables of the reference as TEXT (no Go toolchain is involved):
  /root/reference/bitpacking32_test.go:25-654   (unpack8int32Tests: width, bytes, [8]int32)
  /root/reference/bitpacking64_test.go:25-1744  (unpack8int64Tests: width, bytes, [8]int64)
and writes the (width, data, values) triples — data only — to
  tests/golden/bitpack32_kat.json, tests/golden/bitpack64_kat.json.

Run once in the build container:  python tests/golden/make_bitpack_kat.py
"""
import json
import os
import re
import sys

REF = os.environ.get("PQ_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))

ENTRY = re.compile(
    r"\{\s*(\d+)\s*,\s*\[\]byte\{([^}]*)\}\s*,\s*\[8\]int(32|64)\{([^}]*)\}\s*,?\s*\}",
    re.S,
)


def extract(path, bits):
    text = open(path).read()
    out = []
    for m in ENTRY.finditer(text):
        width = int(m.group(1))
        if int(m.group(3)) != bits:
            continue
        data = [int(x, 0) for x in m.group(2).replace("\n", " ").split(",") if x.strip()]
        values = [int(x) for x in m.group(4).replace("\n", " ").split(",") if x.strip()]
        assert len(values) == 8, (path, m.group(0))
        assert len(data) == width, (path, width, len(data))
        out.append({"width": width, "data": data, "values": values})
    return out


def main():
    for bits, name in ((32, "bitpacking32_test.go"), (64, "bitpacking64_test.go")):
        src = os.path.join(REF, name)
        if not os.path.exists(src):
            sys.exit(f"reference file {src} not found")
        kat = extract(src, bits)
        dst = os.path.join(HERE, f"bitpack{bits}_kat.json")
        with open(dst, "w") as f:
            json.dump({"source": f"{name} (reference test table)", "vectors": kat}, f)
        print(f"{dst}: {len(kat)} vectors, widths {sorted(set(k['width'] for k in kat))}")


if __name__ == "__main__":
    main()
