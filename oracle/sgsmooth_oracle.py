"""oracle/sgsmooth_oracle.py -- TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of the reference's online Savitzky-Golay smoother
CPSNWhere_SGSmooth (psn_where/PSNWhere_SGSmooth.cpp): CalculateQ :133-224,
Insert :91-103, Smoothing :226-272, Filter :274-287 -- IEEE double in the
reference's summation orders. Pinned bit-for-bit against the reference itself
(oracle/_ref/libsgsmooth_ref.so, built from the reference's own source by
oracle/Makefile `ref`) in tests/test_sgsmooth.py.
"""
from __future__ import annotations

import ctypes
import math
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
REF_LIB = os.path.join(_HERE, "_ref", "libsgsmooth_ref.so")


def calculate_q(w: int, degree: int = 1):
    """(Qbegin [hf*w], Qmid [w], Qend [hf*w]) as CalculateQ computes them."""
    hf = (w - 1) // 2
    cols = degree + 1
    qmid = [1.0 / float(w)] * w
    V = [1.0] * (w * cols)
    for order in range(1, degree + 1):
        pos = order
        for t in range(-hf, hf + 1):
            V[pos] = math.pow(float(t), float(order))
            pos += cols
    Q = [0.0] * (w * cols)
    for c in range(cols):
        proj = [0.0] * c
        for r in range(w):
            pos = r * cols + c
            Q[pos] = V[pos]
            for p in range(c):
                proj[p] += Q[r * cols + p] * V[pos]
        norm = 0.0
        for r in range(w):
            pos = r * cols + c
            for p in range(c):
                Q[pos] -= proj[p] * Q[r * cols + p]
            norm += Q[pos] * Q[pos]
        norm = math.sqrt(norm)
        for r in range(w):
            Q[r * cols + c] /= norm
    qb = [0.0] * (hf * w)
    qe = [0.0] * (hf * w)
    front, back, pos = 0, (hf + 1) * cols, 0
    for r in range(hf):
        pq = 0
        for c in range(w):
            for e in range(cols):
                qb[pos] += Q[pq] * Q[front + e]
                qe[pos] += Q[pq] * Q[back + e]
                pq += 1
            pos += 1
        front += cols
        back += cols
    return qb, qmid, qe


class SGSmooth:
    """CPSNWhere_SGSmooth(span, degree): insert() returns refreshPos; .smoothed."""

    def __init__(self, span: int = 9, degree: int = 1):
        self.span, self.degree = span, degree
        self.data: list[float] = []
        self.smoothed: list[float] = []
        self.qrows = 0
        self.q = None

    def _filter(self, coeff, start):
        out = []
        for dp0 in range(start, len(self.data)):
            acc, dp = 0.0, dp0
            for c in range(len(coeff)):
                if dp < 0:
                    break
                acc += coeff[c] * self.data[dp]
                dp -= 1
            out.append(acc)
        return out

    def insert(self, v: float) -> int:
        self.data.append(float(v))
        n = len(self.data)
        w = min(self.span, n)
        w -= (w + 1) % 2
        if w <= self.degree:
            refresh = len(self.smoothed)
            self.smoothed.extend(self.data[len(self.smoothed):])
            return refresh
        hf = (w - 1) // 2
        refresh = 0
        if self.qrows != w:
            self.qrows = w
            self.q = calculate_q(w, self.degree)
            qb, qm, qe = self.q
            sm = []
            pos = 0
            for _ in range(hf):
                acc = 0.0
                for c in range(w):
                    acc += qb[pos] * self.data[c]
                    pos += 1
                sm.append(acc)
            self.smoothed = sm + self._filter(qm, 0)[w - 1:]
        else:
            qb, qm, qe = self.q
            refresh = len(self.smoothed) - hf
            mid = self._filter(qm, len(self.smoothed))
            del self.smoothed[refresh:]
            self.smoothed.extend(mid)
        qe = self.q[2]
        pos = 0
        for _ in range(hf):
            acc = 0.0
            for c in range(n - w, n):
                acc += qe[pos] * self.data[c]
                pos += 1
            self.smoothed.append(acc)
        return refresh


def ref_lib():
    """The reference's own CPSNWhere_SGSmooth (None when _ref was not built)."""
    if not os.path.exists(REF_LIB):
        return None
    L = ctypes.CDLL(REF_LIB)
    L.sgref_create.restype = ctypes.c_void_p
    L.sgref_create.argtypes = [ctypes.c_int, ctypes.c_int]
    L.sgref_destroy.argtypes = [ctypes.c_void_p]
    L.sgref_insert.argtypes = [ctypes.c_void_p, ctypes.c_double]
    L.sgref_size.argtypes = [ctypes.c_void_p]
    L.sgref_result.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.sgref_result.restype = ctypes.c_double
    dp = ctypes.POINTER(ctypes.c_double)
    L.sgref_q.argtypes = [ctypes.c_int, ctypes.c_int, dp, dp, dp]
    return L
