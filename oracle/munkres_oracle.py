"""oracle/munkres_oracle.py -- TEST INFRASTRUCTURE ONLY.

Plain-Python restatement of the reference's Hungarian matcher,
CPSNWhere_Hungarian (psn_where/helpers/PSNWhere_Hungarian.cpp), as
Track2D_MatchingAndUpdating drives it (psn_where/PSNWhere_Tracker2D.cpp
:1040-1064): Initialize (the std::vector<float> overload Tracker2D calls, :67-89, from PSNWhere_Tracker2D.cpp:1059) + Match (:212-359) with its infinity
pre/post-processing (:711-747), the minimum line cover that sizes the padding
(:677-709) and Munkres steps 1-6 (:405-675). Every cost operation is float32
as in the reference (numpy float32 scalars/arrays, IEEE single rounding per
operation), the zero tests are exact, and every scan is in the reference's
row-major order -- so ties break as the reference breaks them.

The reference file itself is not compiled here: it calls MSVC CRT functions
(_isnanf, _finitef) that this image does not provide, and stand-ins for them
are not written. Parity with it is therefore pinned by
this restatement's line-by-line reading only; it is checked against an
exhaustive minimum on integer-valued matrices (tests/test_tracker2d.py).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
FLT_MAX = np.finfo(np.float32).max
NONE, STAR, PRIME = 0, 1, 2


def _step2(P):
    """:426-458: star the first uncovered zero of every row (row-major); covers cleared."""
    n = P.shape[1]
    M = np.zeros((n, n), np.int8)
    rc, cc = np.zeros(n, bool), np.zeros(n, bool)
    for r in range(n):
        for c in range(n):
            if P[r, c] == F32(0) and not rc[r] and not cc[c]:
                M[r, c] = STAR
                rc[r] = cc[c] = True
    return M, np.zeros(n, bool), np.zeros(n, bool)


def _step3(M):
    """:465-480: cover every column holding a star; True when all n columns are covered."""
    cc = (M == STAR).any(axis=0)
    return cc, int(cc.sum()) == M.shape[1]


def _step4(P, M, rc, cc):
    """:491-544: prime uncovered zeros (first in row-major order each time). A prime
    in a row with a star covers the row and uncovers the star's column. Returns
    (row, col) of a prime with no star in its row (step 5), or None (step 6)."""
    n = P.shape[1]
    while True:
        hit = None
        for r in range(n):
            if rc[r]:
                continue
            for c in range(n):
                if P[r, c] == F32(0) and not cc[c]:
                    hit = (r, c)
                    break
            if hit:
                break
        if hit is None:
            return None
        r, c = hit
        M[r, c] = PRIME
        stars = np.nonzero(M[r] == STAR)[0]
        if len(stars):
            rc[r] = True
            cc[stars] = False
        else:
            return hit


def _step5(M, r0, c0):
    """:557-631: the alternating prime/star path from (r0, c0); stars on it are
    unstarred, primes starred; primes erased, covers cleared."""
    n = M.shape[0]
    path = [(r0, c0)]
    while True:
        col = path[-1][1]
        rows = np.nonzero(M[:, col] == STAR)[0]
        if not len(rows):
            break
        r = int(rows[0])
        path.append((r, col))
        primes = np.nonzero(M[r] == PRIME)[0]
        path.append((r, int(primes[0]) if len(primes) else 0))
    for r, c in path:
        M[r, c] = NONE if M[r, c] == STAR else STAR
    M[M == PRIME] = NONE
    return np.zeros(n, bool), np.zeros(n, bool)


def _step6(P, rc, cc):
    """:639-675: the minimum uncovered value is added to covered rows and subtracted
    from uncovered columns (one float32 bias per entry: row bias + column bias)."""
    n = P.shape[0]
    fmin = F32(np.inf)
    for r in range(n):
        if rc[r]:
            continue
        for c in range(n):
            if not cc[c] and P[r, c] < fmin:
                fmin = P[r, c]
    for r in range(n):
        rb = fmin if rc[r] else F32(0)
        for c in range(n):
            cb = -fmin if not cc[c] else F32(0)
            P[r, c] = F32(P[r, c] + F32(rb + cb))


def _min_line_cover(E):
    """:677-709: the deficiency of the zero pattern of E (steps 2, 3, 4 once)."""
    n = E.shape[1]
    M, rc, cc = _step2(E)
    cc, _ = _step3(M)
    _step4(E, M, rc, cc)
    return n - int(rc.sum() + cc.sum())


def hungarian_match(cost):
    """CPSNWhere_Hungarian Initialize(std::vector<float>, rows, cols) (:67-89) + Match() -> (rows, cols,
    match costs) of the matched pairs in row-major order, as stMatchInfo holds them.
    An empty matrix, or one holding a NaN (:78-81), matches nothing."""
    C = np.array(cost, np.float32, copy=True)
    R, K = C.shape
    if R * K == 0 or np.isnan(C).any():
        return [], [], []
    # CostMatrixPreprocessing (:711-735): non-finite -> FLT_MAX - (float sum of the finite costs)
    finite = np.isfinite(C)
    s = F32(0)
    for r in range(R):
        for c in range(K):
            if finite[r, c]:
                s = F32(s + C[r, c])
    repl = F32(FLT_MAX - s)
    C[~finite] = repl
    xcon = [r for r in range(R) if finite[r].any()]
    ycon = [c for c in range(K) if finite[:, c].any()]
    n = max(R, K)
    P = np.zeros((n, n), np.float32)
    P[:R, :K] = C
    E = np.full((n, n), np.inf, np.float32)
    pmax = F32(0)
    for r in range(n):
        for c in range(n):
            if np.isfinite(P[r, c]):
                E[r, c] = F32(0)
                if P[r, c] > pmax:
                    pmax = P[r, c]
    n += _min_line_cover(E)
    P = np.full((n, n), pmax, np.float32)
    for i, r in enumerate(xcon):
        for j, c in enumerate(ycon):
            P[i, j] = C[r, c]
    # step 1 (:405-419): subtract each row's minimum (rows whose minimum is 0 or inf are left)
    for r in range(n):
        m = P[r].min()
        if m == F32(0) or m == F32(np.inf):
            continue
        P[r] = P[r] - m
    M, rc, cc = _step2(P)
    while True:
        cc, done = _step3(M)
        if done:
            break
        while True:
            hit = _step4(P, M, rc, cc)
            if hit is not None:
                rc, cc = _step5(M, *hit)
                break
            _step6(P, rc, cc)
    # MatchResultPostProcessing (:737-747) and the extraction loop (:339-354)
    C[C == repl] = np.inf
    rows, cols, costs = [], [], []
    for r in range(R):
        for c in range(K):
            if M[r, c] == STAR and np.isfinite(C[r, c]):
                rows.append(r)
                cols.append(c)
                costs.append(F32(C[r, c]))
    return rows, cols, costs


def assign(cost) -> list:
    """Track2D_MatchingAndUpdating's assignment (:1040-1064): non-finite costs ->
    max(finite, -1000) + 100 (float32), the Hungarian, and pairs at that
    substitute cost dropped. Returns the tracker index per detection or -1."""
    c = np.array(cost, np.float32, copy=True).reshape(np.shape(cost))
    D = c.shape[0]
    match = [-1] * D
    if c.size == 0:
        return match
    max_cost = F32(-1000.0)
    for v in c.ravel():
        if np.isfinite(v) and max_cost < v:
            max_cost = v
    max_cost = F32(max_cost + F32(100.0))
    c[~np.isfinite(c)] = max_cost
    rows, cols, costs = hungarian_match(c)
    for r, k, v in zip(rows, cols, costs):
        if max_cost == v:
            continue
        match[r] = k
    return match
