"""CPU model of the repair plan's Gauss-Jordan fast path (decds_amd/csrc/rlnc_kernels.hip plan_fast), step
for step in the kernel's own integer arithmetic — exp table of three periods (765 bytes) with zeros after
it, log 0 = PLAN_LOG0 = 1024, unreduced log sums — against the incremental rank test of chunkset.rs:173-184
restated here and the oracle's matrix inverse. Pins what the kernel relies on: every exp index stays
inside the 2304-byte table, a zero factor or entry reads a zero product, row swaps at zero pivots, the
give-up on a dependent first ten, and the verdicts of the candidates after the ten. (The kernel itself
is compared with the oracle on the GPU: tests/test_gpu_parity.py::test_repair_plan_fast_path_matches_oracle.)"""
import numpy as np

import oracle as o

K, N, LOG0, EXP_VALID, EXP_BYTES = 10, 16, 1024, 765, 2304


def _tables(poly=o.POLY, gen=2):
    exp, lg, x = [0] * EXP_BYTES, [0] * 256, 1
    for i in range(255):
        exp[i] = exp[i + 255] = exp[i + 510] = x
        lg[x] = i
        x = o.gf_mul(x, gen, poly)
    lg[0] = LOG0
    return exp, lg


EXP, LOG = _tables()


def fast_plan(vecs, cand):
    """plan_fast: (sel, rank, input-major inverse, verdicts), or None where the kernel hands over"""
    if any(int(c) >= N for c in cand[:K]):
        return None
    M = [[int(vecs[cand[i]][c]) if c < K else int(c == K + i) for c in range(2 * K)] for i in range(K)]
    LM = [[LOG[v] for v in row] for row in M]
    for s in range(K):
        f = [LM[i][s] for i in range(K)]
        if f[s] == LOG0:
            q = next((j for j in range(s + 1, K) if f[j] != LOG0), None)
            if q is None:
                return None
            M[s], M[q], LM[s], LM[q], f[s], f[q] = M[q], M[s], LM[q], LM[s], f[q], f[s]
        u = 255 - f[s]
        for i in range(K):
            idx = [x + u + (0 if i == s else f[i]) for x in LM[s]]
            assert max(idx) < EXP_BYTES
            assert all((x < EXP_VALID) == (x < LOG0) for x in idx)  # nonzero products in the table's periods
            M[i] = [EXP[x] for x in idx] if i == s else [a ^ EXP[x] for a, x in zip(M[i], idx)]
        LM = [[LOG[v] for v in row] for row in M]
    inv = [0] * (K * K)
    for s in range(K):
        assert M[s][:K] == [int(c == s) for c in range(K)]
        for k in range(K):
            inv[k * K + s] = M[s][K + k]
    ver, a = [0] * K + [-1] * (N - K), K
    while a < N and cand[a] < N:
        ver[a] = 3
        a += 1
    return [int(c) for c in cand[:K]], K, inv, ver


def incremental_plan(vecs, cand):
    """the rank test in arrival order (chunkset.rs:173-184): accepted iff it raises the rank"""
    basis, sel, ver = [], [], [-1] * N
    for a in range(N):
        r = int(cand[a])
        if r >= N:
            break
        if len(sel) == K:
            ver[a] = 3
            continue
        v = [int(x) for x in vecs[r]]
        for p, b in basis:
            if v[p]:
                v = [x ^ o.gf_mul(v[p], y) for x, y in zip(v, b)]
        nz = [i for i in range(K) if v[i]]
        if not nz:
            ver[a] = 4
            continue
        p = nz[0]
        iv = o.gf_inv(v[p])
        v = [o.gf_mul(iv, x) for x in v]
        basis = [(pp, [x ^ o.gf_mul(b[p], y) for x, y in zip(b, v)]) for pp, b in basis] + [(p, v)]
        sel.append(r)
        ver[a] = 0
    if len(sel) < K:
        return sel, len(sel), None, ver
    inv_m = o.matrix_inverse(np.array([[int(x) for x in vecs[r]] for r in sel], np.uint8))
    return sel, K, [int(inv_m[i][k]) for k in range(K) for i in range(K)], ver


def test_fast_path_equals_the_incremental_plan():
    rng = np.random.default_rng(1)
    taken = given_up = 0
    for t in range(500):
        kind = t % 5
        if kind == 0:
            vecs = rng.integers(0, 256, (N, K), dtype=np.uint8)
        elif kind == 1:  # permuted scaled unit vectors: a zero pivot at most columns
            vecs = rng.integers(0, 256, (N, K), dtype=np.uint8)
            vecs[:K] = 0
            vecs[np.arange(K), rng.permutation(K)] = rng.integers(1, 256, K)
        elif kind == 2:
            vecs = (rng.integers(0, 256, (N, K)) * (rng.random((N, K)) < 0.25)).astype(np.uint8)
        elif kind == 3:
            vecs = rng.integers(0, 4, (N, K), dtype=np.uint8)
        else:  # the first ten dependent
            vecs = rng.integers(0, 256, (N, K), dtype=np.uint8)
            vecs[3] = [o.gf_mul(7, int(x)) ^ int(y) for x, y in zip(vecs[1], vecs[2])]
        length = N if t % 3 == 0 else int(rng.integers(0, N + 1))
        ids = rng.permutation(N)[:length] if t % 2 == 0 else rng.integers(0, N, length)
        cand = np.full(N, 0xFF, np.uint8)
        cand[:length] = ids
        want, got = incremental_plan(vecs, cand), fast_plan(vecs, cand)
        if got is None:
            given_up += 1
            continue
        taken += 1
        assert got == want, t
    assert taken > 50 and given_up > 50


def test_incremental_restatement_matches_the_oracle_decoder():
    """the incremental restatement above against oracle.Decoder's verdicts (the plan tests' reference)"""
    rng = np.random.default_rng(2)
    for t in range(40):
        vecs = rng.integers(0, 3 if t % 2 else 256, (N, K), dtype=np.uint8)
        cand = rng.integers(0, N, N).astype(np.uint8)
        d = o.Decoder(3, K)
        ok = []
        for r in cand:
            ok.append(not d.is_already_decoded() and d.decode(np.concatenate([vecs[r], np.zeros(3, np.uint8)])) == o.OK)
        _, rank, _, mine = incremental_plan(vecs, cand)
        assert rank == d.rank()
        assert [v == 0 for v in mine] == ok, t
