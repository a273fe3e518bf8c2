"""The field/marker identification procedure (tools/identify_field.py) recovers the
polynomial and boundary marker from one coded chunk framed as a decds share file."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import identify_field as idf  # noqa: E402
import oracle as o  # noqa: E402


def varint(v):
    if v < 251:
        return bytes([v])
    if v < 1 << 16:
        return b"\xfb" + v.to_bytes(2, "little")
    if v < 1 << 32:
        return b"\xfc" + v.to_bytes(4, "little")
    return b"\xfd" + v.to_bytes(8, "little")


def test_thirty_irreducible_polynomials():
    polys = idf.irreducible_polys()
    assert len(polys) == 30 and 0x11D in polys and 0x11B in polys


@pytest.mark.parametrize("poly,marker", [(0x11D, 0x81), (0x11B, 0x81), (0x14D, 0x01), (0x11D, 0xFF)])
def test_identify_from_share_file(poly, marker, tmp_path):
    data = o.fill_random(poly * 7 + marker, o.CS)
    cv = o.fill_random(99, 10)
    cv[9] |= 1
    coded = o.code_with_coding_vector(data, cv, poly=poly, marker=marker)
    share = varint(3) + varint(3 * 16 + 5) + varint(coded.size) + coded.tobytes() + varint(0)
    cs_id, chunk_id, parsed = idf.parse_share(share)
    assert (cs_id, chunk_id) == (3, 53) and np.array_equal(parsed, coded)
    hits, m = idf.identify(parsed, data)
    assert hits == [poly] and m == marker
