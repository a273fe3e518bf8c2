"""Re-pin the two rlnc 0.4.0 constants this codec could only recall (GF(2^8) polynomial, boundary
marker) from ONE reference-produced coded chunk and the chunkset it came from.

A decds share file (`chunkset.N/shareXX.data`, decds-bin handle_break.rs:67-106) is a bincode
`standard()` (consts.rs:2) serialisation of ProofCarryingChunk (chunk.rs:52-55):
  chunkset_id: varint, chunk_id: varint, erasure_coded_data: Vec<u8> (varint length + bytes), proof.
Its erasure-coded data is the rlnc full coded piece: 10-byte coding vector c || payload y with
y[col] = sum_i c_i * piece_i[col]. Columns below 1,048,567 involve data bytes only, so they
identify the polynomial among the 30 irreducible degree-8 candidates; column 1,048,567 of piece 9
holds the marker m, which y then determines as m = (y - sum_{i<9} c_i*piece_i) / c_9.

Layout hypotheses (identify_layout): the coding vector before or after the payload, and the marker
right after the data (then zeros), at the very end of the padding, or absent; each fit is reported
with its polynomial and marker, so an unexpected layout is named instead of reported as "no
polynomial".

usage: python tools/identify_field.py SHARE_FILE CHUNKSET_DATA_FILE
       (CHUNKSET_DATA_FILE = the 10 MiB chunkset, e.g. decds-bin's chunkset.N.data, zero-padded)
"""
import json
import os
import sys

import numpy as np

K, CS = 10, 10 * (1 << 20)
L = (CS + 1 + K - 1) // K


def irreducible_polys():
    """the 30 irreducible polynomials of degree 8 over GF(2), as 9-bit integers"""
    def mod(a, b):
        db = b.bit_length()
        while a.bit_length() >= db:
            a ^= b << (a.bit_length() - db)
        return a
    return [p for p in range(0x100, 0x200) if p & 1 and all(mod(p, q) for q in range(2, 32))]


def gf_mul_table(poly):
    # the checker's product table (oracle/, test infrastructure) for each candidate polynomial
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle
    return oracle.mul_table(poly)


def read_varint(buf, pos):
    """bincode 2 standard-config unsigned varint"""
    b = buf[pos]
    if b < 251:
        return b, pos + 1
    width = {251: 2, 252: 4, 253: 8, 254: 16}[b]
    return int.from_bytes(buf[pos + 1:pos + 1 + width], "little"), pos + 1 + width


def parse_share(buf):
    cs_id, p = read_varint(buf, 0)
    chunk_id, p = read_varint(buf, p)
    n, p = read_varint(buf, p)
    return cs_id, chunk_id, np.frombuffer(buf[p:p + n], np.uint8)


# layout hypotheses the re-pin tries: where the 10-byte coding vector sits in the full
# coded piece, and where Encoder::new puts the boundary marker in the padded pieces
PREFIXES = ("cv||payload", "payload||cv")
MARKERS = ("marker-then-zeros", "zeros-then-marker", "no-marker")


def split_piece(coded, prefix):
    coded = np.asarray(coded, np.uint8)
    return (coded[:K], coded[K:]) if prefix == "cv||payload" else (coded[-K:], coded[:-K])


def _polys_for(cv, y, data, cols):
    pieces = np.stack([data[i * L + cols] if i < 9 else data[np.minimum(9 * L + cols, CS - 1)] for i in range(K)])
    hits = []
    for p in irreducible_polys():
        t = gf_mul_table(p)
        acc = np.zeros(len(cols), np.uint8)
        for i in range(K):
            acc ^= t[cv[i], pieces[i]]
        if np.array_equal(acc, y[cols]):
            hits.append(p)
    return hits


def _marker_for(cv, y, data, poly, placement):
    """the marker value under `placement`, or None if the tail columns contradict it. Piece 9 holds
    data bytes up to column CS - 9L, then the padding; the other pieces are data only."""
    t = gf_mul_table(poly)
    first = CS - 9 * L                             # piece 9's first padding column
    mcol = {"marker-then-zeros": first, "zeros-then-marker": L - 1, "no-marker": None}[placement]
    inv = next(b for b in range(1, 256) if t[cv[9], b] == 1) if cv[9] else None
    marker = None
    for col in range(first, L):
        rest = 0
        for i in range(9):
            rest ^= int(t[cv[i], data[i * L + col]])
        got = int(y[col]) ^ rest                   # = cv[9] * piece9[col]
        if col == mcol:
            if inv is None:
                return None
            marker = int(t[inv, got])
            if marker == 0:
                return None                        # a zero "marker" is the no-marker layout
        elif got != 0:
            return None
    return marker if mcol is not None else "none"


def identify_layout(coded, chunkset, probe_cols=64):
    """every (prefix, marker placement) hypothesis the chunk is consistent with:
    [{"prefix", "marker_placement", "polynomials", "marker"}]; empty = no known layout fits"""
    data = np.asarray(chunkset, np.uint8)
    rng = np.random.default_rng(0)
    cols = rng.choice(L - 10, size=min(probe_cols, L - 10), replace=False)
    out = []
    for prefix in PREFIXES:
        cv, y = split_piece(coded, prefix)
        hits = _polys_for(cv, y, data, cols)
        for placement in MARKERS:
            for p in hits:
                m = _marker_for(cv, y, data, p, placement)
                if m is not None:
                    out.append({"prefix": prefix, "marker_placement": placement, "polynomial": p,
                                "marker": None if m == "none" else m})
    return out


def identify(coded, chunkset, probe_cols=64):
    """the recalled layout only (cv || payload, marker then zeros): (polys consistent with the data
    columns, marker or None)"""
    cv, y = split_piece(coded, "cv||payload")
    data = np.asarray(chunkset, np.uint8)
    rng = np.random.default_rng(0)
    cols = rng.choice(L - 10, size=min(probe_cols, L - 10), replace=False)
    hits = _polys_for(cv, y, data, cols)
    marker = None
    if len(hits) == 1:
        m = _marker_for(cv, y, data, hits[0], "marker-then-zeros")
        marker = m if isinstance(m, int) else None
    return hits, marker


def main():
    share, data_file = sys.argv[1], sys.argv[2]
    buf = open(share, "rb").read()
    cs_id, chunk_id, coded = parse_share(buf)
    data = np.fromfile(data_file, np.uint8)
    if data.size < CS:
        data = np.concatenate([data, np.zeros(CS - data.size, np.uint8)])
    fits = identify_layout(coded, data[:CS])
    print(json.dumps({"chunkset_id": cs_id, "chunk_id": chunk_id,
                      "layouts": [dict(f, polynomial=hex(f["polynomial"]),
                                       marker=None if f["marker"] is None else hex(f["marker"])) for f in fits],
                      "verdict": ("no known layout fits: not an rlnc-0.4.0-style piece of this chunkset under any "
                                  "hypothesis tried (%s x %s)" % (PREFIXES, MARKERS)) if not fits else
                                 ("pinned" if len(fits) == 1 else "ambiguous")}))


if __name__ == "__main__":
    main()
