"""The levels -> nesting restatement (oracle.nest_levels) against the reference's
record-shredding known answers (tests/golden/dremel_kat.json from data_store_test.go:18-497): for
every leaf column, the list offsets / presence per repetition level and the leaf validity computed
from the asserted levels must describe exactly the records the reference reads back."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "dremel_kat.json")))


def rep_def_of(schema, path):
    """Definition level of each REPEATED node on `path` (readColumnSchema, schema.go:893-990)."""
    reps = dict(schema)
    parts = path.split(".")
    d, out = 0, []
    for k in range(1, len(parts) + 1):
        rep = reps[".".join(parts[:k])]
        if rep != "REQUIRED":
            d += 1
        if rep == "REPEATED":
            out.append(d)
    return out


def expect_from_rows(rows, schema, path):
    """Walk the records the reference returns along `path`: per repeated node one list per enclosing
    instance (present iff its parent object exists; an absent key is an empty list), per leaf slot
    non-null iff the value exists."""
    reps = dict(schema)
    parts = path.split(".")
    chain = [(parts[k], reps[".".join(parts[:k + 1])]) for k in range(len(parts))]
    nlev = sum(1 for _, r in chain if r == "REPEATED")
    lists = [([], []) for _ in range(nlev)]
    leaf_valid, values = [], []

    def visit(obj, j, lvl):
        if j == len(chain):
            leaf_valid.append(obj is not None)
            if obj is not None:
                values.append(obj)
            return
        name, rep = chain[j]
        child = obj.get(name) if isinstance(obj, dict) else None
        if rep == "REPEATED":
            lists[lvl][0].append(obj is not None)
            items = child if child is not None else []
            lists[lvl][1].append(len(items))
            for it in items:
                visit(it, j + 1, lvl + 1)
        else:
            visit(child, j + 1, lvl)

    for row in rows:
        visit(row, 0, 0)
    levels = [(np.concatenate([[0], np.cumsum(c)]).astype(np.int32), np.array(v, np.uint8)) for v, c in lists]
    return levels, np.array(leaf_valid, np.uint8), values


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_nesting_matches_reference_records(kat):
    for lf in kat["leaves"]:
        rd = rep_def_of(kat["schema"], lf["path"])
        assert len(rd) == lf["max_rep"]
        levels, leaf_valid = O.nest_levels(lf["def"], lf["rep"], lf["max_def"], rd)
        want_levels, want_leaf, want_values = expect_from_rows(kat["rows"], kat["schema"], lf["path"])
        assert want_values == lf["values"], f"{kat['name']} {lf['path']}: transcription"
        assert len(levels) == len(want_levels)
        for (o, v), (wo, wv) in zip(levels, want_levels):
            np.testing.assert_array_equal(o, wo, err_msg=f"{kat['name']} {lf['path']} offsets")
            np.testing.assert_array_equal(v, wv, err_msg=f"{kat['name']} {lf['path']} validity")
        np.testing.assert_array_equal(leaf_valid, want_leaf, err_msg=f"{kat['name']} {lf['path']} leaf")
        assert int(leaf_valid.sum()) == len(lf["values"])
