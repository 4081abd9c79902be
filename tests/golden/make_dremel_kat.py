"""Writes dremel_kat.json: the record-shredding known-answer tests of the reference,
data_store_test.go:18-497 (TestOneColumn ... TestZeroRL), transcribed as data: the schema (path +
repetition of every node), the records the reference reads back (row.getData() must equal them),
and per leaf column the definition levels, repetition levels and values the reference asserts.
Pins the levels -> nesting restatement (oracle.nest_levels) against the reference's own records.

  python tests/golden/make_dremel_kat.py
"""
import json
import os

R, O, P = "REQUIRED", "OPTIONAL", "REPEATED"


def leaf(path, max_def, max_rep, d, r, values):
    return {"path": path, "max_def": max_def, "max_rep": max_rep, "def": d, "rep": r, "values": values}


LANG_ROW = {"Name": [{"Language": [{"Code": 1, "Country": 100}, {"Code": 2}], "URL": 10},
                     {"URL": 11},
                     {"Language": [{"Code": 3, "Country": 101}]}]}

KATS = [
    {"name": "TestOneColumn", "source": "data_store_test.go:18-46",
     "schema": [["DocID", R]],
     "rows": [{"DocID": 10}, {"DocID": 20}],
     "leaves": [leaf("DocID", 0, 0, [0, 0], [0, 0], [10, 20])]},
    {"name": "TestOneColumnOptional", "source": "data_store_test.go:48-74",
     "schema": [["DocID", O]],
     "rows": [{"DocID": 10}, {}],
     "leaves": [leaf("DocID", 1, 0, [1, 0], [0, 0], [10])]},
    {"name": "TestOneColumnRepeated", "source": "data_store_test.go:76-102",
     "schema": [["DocID", P]],
     "rows": [{"DocID": [10, 20]}, {}],
     "leaves": [leaf("DocID", 1, 1, [1, 1, 0], [0, 1, 0], [10, 20])]},
    {"name": "TestComplexPart1", "source": "data_store_test.go:104-177",
     "schema": [["Name", P], ["Name.Language", P], ["Name.Language.Code", R], ["Name.Language.Country", O],
                ["Name.URL", O]],
     "rows": [LANG_ROW],
     "leaves": [leaf("Name.Language.Code", 2, 2, [2, 2, 1, 2], [0, 2, 1, 1], [1, 2, 3]),
                leaf("Name.Language.Country", 3, 2, [3, 2, 1, 3], [0, 2, 1, 1], [100, 101]),
                leaf("Name.URL", 2, 1, [2, 2, 1], [0, 1, 1], [10, 11])]},
    {"name": "TestComplexPart2", "source": "data_store_test.go:179-225",
     "schema": [["Links", O], ["Links.Backward", P], ["Links.Forward", P]],
     "rows": [{"Links": {"Forward": [20, 40, 60]}}, {"Links": {"Backward": [10, 30], "Forward": [80]}}],
     "leaves": [leaf("Links.Forward", 2, 1, [2, 2, 2, 2], [0, 1, 1, 0], [20, 40, 60, 80]),
                leaf("Links.Backward", 2, 1, [1, 2, 2], [0, 0, 1], [10, 30])]},
    {"name": "TestComplex", "source": "data_store_test.go:227-344",
     "schema": [["DocId", R], ["Links", O], ["Links.Backward", P], ["Links.Forward", P], ["Name", P],
                ["Name.Language", P], ["Name.Language.Code", R], ["Name.Language.Country", O], ["Name.URL", O]],
     "rows": [dict(DocId=10, Links={"Forward": [20, 40, 60]}, **LANG_ROW),
              {"DocId": 20, "Links": {"Backward": [10, 30], "Forward": [80]}, "Name": [{"URL": 12}]}],
     "leaves": [leaf("DocId", 0, 0, [0, 0], [0, 0], [10, 20]),
                leaf("Name.URL", 2, 1, [2, 2, 1, 2], [0, 1, 1, 0], [10, 11, 12]),
                leaf("Links.Forward", 2, 1, [2, 2, 2, 2], [0, 1, 1, 0], [20, 40, 60, 80]),
                leaf("Links.Backward", 2, 1, [1, 2, 2], [0, 0, 1], [10, 30]),
                leaf("Name.Language.Country", 3, 2, [3, 2, 1, 3, 1], [0, 2, 1, 1, 0], [100, 101]),
                leaf("Name.Language.Code", 2, 2, [2, 2, 1, 2, 1], [0, 2, 1, 1, 0], [1, 2, 3])]},
    {"name": "TestTwitterBlog", "source": "data_store_test.go:346-389",
     "schema": [["level1", P], ["level1.level2", P]],
     "rows": [{"level1": [{"level2": [1, 2, 3]}, {"level2": [4, 5, 6, 7]}]},
              {"level1": [{"level2": [8]}, {"level2": [9, 10]}]}],
     "leaves": [leaf("level1.level2", 2, 2, [2] * 10, [0, 2, 2, 1, 2, 2, 2, 0, 1, 2], list(range(1, 11)))]},
    {"name": "TestEmptyParent", "source": "data_store_test.go:391-427",
     "schema": [["baz", O], ["baz.list", P], ["baz.list.element", R]],
     "rows": [{"baz": {}}],
     "leaves": [leaf("baz.list.element", 2, 1, [1], [0], [])]},
    {"name": "TestZeroRL", "source": "data_store_test.go:429-474",
     "schema": [["baz", R], ["baz.list", P], ["baz.list.element", R], ["baz.list.element.quux", R]],
     "rows": [{"baz": {"list": [{"element": {"quux": 23}}, {"element": {"quux": 42}}]}}],
     "leaves": [leaf("baz.list.element.quux", 1, 1, [1, 1], [0, 1], [23, 42])]},
    {"name": "TestZeroRL/optional", "source": "data_store_test.go:476-496",
     "schema": [["baz", R], ["baz.list", P], ["baz.list.element", R], ["baz.list.element.quux", O]],
     "rows": [{"baz": {"list": [{"element": {"quux": 23}}, {"element": {"quux": 42}}]}}],
     "leaves": [leaf("baz.list.element.quux", 2, 1, [2, 2], [0, 1], [23, 42])]},
]

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "dremel_kat.json")
    with open(out, "w") as f:
        json.dump(KATS, f, indent=1)
    print(out, len(KATS))
