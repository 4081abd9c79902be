"""Pin the CPU oracle against the reference's own known-answer vectors (CPU only)."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


def _kat(bits):
    with open(os.path.join(GOLDEN, f"bitpack{bits}_kat.json")) as f:
        return json.load(f)["vectors"]


@pytest.mark.parametrize("bits", [32, 64])
def test_unpack_kat(orc, bits):
    """unpack8int{32,64}_w vs bitpacking{32,64}_test.go tables (TestUnpack8int32/64)."""
    vecs = _kat(bits)
    assert len(vecs) > (100 if bits == 32 else 300)
    for v in vecs:
        got = orc.unpack8(v["width"], bytes(v["data"]), bits)
        assert got == v["values"], v


@pytest.mark.parametrize("bits", [32, 64])
def test_pack_kat(orc, bits):
    """pack8int{32,64}_w (the reference writer's packer) round-trips the same tables."""
    for v in _kat(bits):
        assert orc.pack8(v["width"], v["values"], bits) == bytes(v["data"]), v
