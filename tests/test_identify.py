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


def _coded_under(data, cv, poly, marker, prefix, placement):
    """a full coded piece built under a layout hypothesis (numpy restatement via the oracle's tables)"""
    t = o.mul_table(poly)
    padded = np.zeros(10 * o.L, np.uint8)
    padded[:o.CS] = data
    if placement == "marker-then-zeros":
        padded[o.CS] = marker
    elif placement == "zeros-then-marker":
        padded[-1] = marker
    y = np.zeros(o.L, np.uint8)
    for i in range(10):
        y ^= t[cv[i], padded[i * o.L:(i + 1) * o.L]]
    return np.concatenate([cv, y] if prefix == "cv||payload" else [y, cv])


@pytest.mark.parametrize("prefix", idf.PREFIXES)
@pytest.mark.parametrize("placement", idf.MARKERS)
def test_identify_layout_names_the_hypothesis(prefix, placement):
    poly, marker = (0x11D, 0x81) if prefix == "cv||payload" else (0x12B, 0x5A)
    data = o.fill_random(len(prefix) * 31 + len(placement), o.CS)
    cv = o.fill_random(7 + len(placement), 10)
    cv[9] |= 1
    coded = _coded_under(data, cv, poly, marker, prefix, placement)
    fits = idf.identify_layout(coded, data)
    want = {"prefix": prefix, "marker_placement": placement, "polynomial": poly,
            "marker": None if placement == "no-marker" else marker}
    assert fits == [want]


def test_identify_layout_reports_nothing_for_unrelated_bytes():
    data = o.fill_random(5, o.CS)
    assert idf.identify_layout(o.fill_random(6, o.F), data) == []
