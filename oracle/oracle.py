"""CPU oracle for the IVF-PQ search path — TEST INFRASTRUCTURE ONLY.

ctypes front-end over ``oracle/liboracle.so`` (built from ``ivfpq_oracle.c``
by ``oracle/Makefile``).  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module; the product
package never does.  See the header of ``ivfpq_oracle.c`` for the restated
reference semantics and how they are pinned.

``OracleIVFPQ`` mirrors the part of ``faiss.IndexIVFPQ`` that Chameleon's
harnesses exercise (``Chameleon/Faiss_experiments/bench_polysemous_1bn.py:
272-291, 343, 430``): train / add / add_with_ids / search /
search_preassigned with ``nprobe``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_f32p = ctypes.POINTER(ctypes.c_float)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u8p = ctypes.POINTER(ctypes.c_uint8)


def build() -> str:
    path = os.path.join(_HERE, "liboracle.so")
    src = os.path.join(_HERE, "ivfpq_oracle.c")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return path


def lib():
    global _LIB
    if _LIB is None:
        _LIB = ctypes.CDLL(build())
        L = _LIB
        L.or_tree.restype = ctypes.c_float
        L.or_tree.argtypes = [_f32p, _f32p, ctypes.c_int, ctypes.c_int]
        L.or_norms.argtypes = [_f32p, ctypes.c_int64, ctypes.c_int, _f32p]
        L.or_coarse_search.argtypes = [_f32p, ctypes.c_int64, ctypes.c_int, _f32p, _f32p, ctypes.c_int,
                                       ctypes.c_int, _i64p, _f32p, ctypes.c_int]
        L.or_coarse_search_metric.argtypes = L.or_coarse_search.argtypes + [ctypes.c_int]
        L.or_ip_table.argtypes = [_f32p, ctypes.c_int64, ctypes.c_int, _f32p, ctypes.c_int, ctypes.c_int, _f32p]
        L.or_linear_transform.argtypes = [_f32p, ctypes.c_int64, ctypes.c_int, _f32p, _f32p, ctypes.c_int, _f32p]
        L.or_precompute_T1.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, _f32p, ctypes.c_int, ctypes.c_int, _f32p]
        L.or_encode.argtypes = [_f32p, ctypes.c_int64, ctypes.c_int, _f32p, _f32p, ctypes.c_int, _f32p,
                                ctypes.c_int, ctypes.c_int, _i64p, _u8p, ctypes.c_int]
        L.or_search_preassigned.argtypes = [_f32p, ctypes.c_int64, ctypes.c_int, _f32p, _f32p, ctypes.c_int,
                                            ctypes.c_int, _i64p, _u8p, _i64p, ctypes.c_int, _i64p, _f32p,
                                            ctypes.c_int, _f32p, _i64p, ctypes.c_int]
        L.or_search_preassigned_metric.argtypes = L.or_search_preassigned.argtypes + [ctypes.c_int, _f32p]
        L.or_kmeans.argtypes = [_f32p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                _f32p, ctypes.c_int]
        L.or_train_ivfpq.argtypes = [_f32p, ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_uint64, _f32p, _f32p, ctypes.c_int]
        L.or_rand_perm_prefix.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64, _i64p]
        L.or_encode_metric.argtypes = L.or_encode.argtypes + [ctypes.c_int]
        L.or_kmeans_metric.argtypes = L.or_kmeans.argtypes + [ctypes.c_int]
        L.or_train_ivfpq_metric.argtypes = L.or_train_ivfpq.argtypes + [ctypes.c_int]
    return _LIB


def _p(a, t):
    return a.ctypes.data_as(t)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def default_threads() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        return os.cpu_count() or 1


# ---- stand-alone restated functions -------------------------------------------------

def tree(x, y, kind: int) -> float:
    """Faiss AVX reduction order; kind 0 = IP, 1 = L2, 2 = norm."""
    x = _f32(x)
    y = _f32(y)
    return float(lib().or_tree(_p(x, _f32p), _p(y, _f32p), x.shape[0], kind))


def norms(x):
    x = _f32(x)
    out = np.empty(x.shape[0], np.float32)
    lib().or_norms(_p(x, _f32p), x.shape[0], x.shape[1], _p(out, _f32p))
    return out


def linear_transform(x, A, b=None):
    """y = x A^T (+ b) in the t-ordered fmaf order (or_linear_transform): OPQ apply."""
    x = _f32(x)
    A = _f32(A)
    d_out, d_in = A.shape
    assert x.shape[1] == d_in
    y = np.empty((x.shape[0], d_out), np.float32)
    bb = None if b is None else _f32(b)
    lib().or_linear_transform(_p(x, _f32p), x.shape[0], d_in, _p(A, _f32p), None if bb is None else _p(bb, _f32p),
                              d_out, _p(y, _f32p))
    return y


def ip_table(x, codebook):
    """T3[q][m][j] = <q_m, C_mj> (ProductQuantizer::compute_inner_prod_table)."""
    x = _f32(x)
    codebook = _f32(codebook)
    M, ksub, _ = codebook.shape
    out = np.empty((x.shape[0], M, ksub), np.float32)
    lib().or_ip_table(_p(x, _f32p), x.shape[0], x.shape[1], _p(codebook, _f32p), M, ksub, _p(out, _f32p))
    return out


def precompute_T1(centroids, codebook):
    centroids = _f32(centroids)
    codebook = _f32(codebook)
    M, ksub, _ = codebook.shape
    nlist, d = centroids.shape
    out = np.empty((nlist, M, ksub), np.float32)
    lib().or_precompute_T1(_p(centroids, _f32p), nlist, d, _p(codebook, _f32p), M, ksub, _p(out, _f32p))
    return out


METRIC_INNER_PRODUCT = 0
METRIC_L2 = 1


def coarse_search(x, centroids, nprobe, nthreads=None, metric=METRIC_L2):
    """IndexFlatL2 / IndexFlatIP search of the centroids: (dis, lists) [n][nprobe]."""
    x = _f32(x)
    centroids = _f32(centroids)
    cn = norms(centroids)
    n, d = x.shape
    nlist = centroids.shape[0]
    nprobe = min(nprobe, nlist)
    lists = np.empty((n, nprobe), np.int64)
    dis = np.empty((n, nprobe), np.float32)
    lib().or_coarse_search_metric(_p(x, _f32p), n, d, _p(centroids, _f32p), _p(cn, _f32p), nlist, nprobe,
                                  _p(lists, _i64p), _p(dis, _f32p), nthreads or default_threads(), metric)
    return dis, lists


def kmeans(x, k, niter, seed, nthreads=None, metric=1):
    x = _f32(x)
    out = np.empty((k, x.shape[1]), np.float32)
    lib().or_kmeans_metric(_p(x, _f32p), x.shape[0], x.shape[1], k, niter, seed, _p(out, _f32p),
                           nthreads or default_threads(), metric)
    return out


def rand_perm_prefix(n, k, seed):
    out = np.empty(k, np.int64)
    lib().or_rand_perm_prefix(n, k, seed, _p(out, _i64p))
    return out


class OracleIVFPQ:
    """CPU IVF-PQ (by_residual; L2 with precomputed tables, or inner product)
    with Faiss-1.7.1 order."""

    def __init__(self, d, nlist, M, nbits=8, metric=METRIC_L2):
        if nbits != 8:
            raise ValueError("oracle supports nbits=8")
        if d % M:
            raise ValueError("d must be a multiple of M")
        self.d, self.nlist, self.M, self.ksub = d, nlist, M, 1 << nbits
        self.nprobe = 1
        self.centroids = None
        self.codebook = None
        self.T1 = None
        self.list_codes = [np.zeros((0, M), np.uint8) for _ in range(nlist)]
        self.list_ids = [np.zeros(0, np.int64) for _ in range(nlist)]
        self.ntotal = 0
        self.nthreads = default_threads()
        self.metric = metric

    @property
    def is_trained(self):
        return self.centroids is not None

    def set_trained(self, centroids, codebook):
        self.centroids = _f32(centroids).reshape(self.nlist, self.d)
        self.codebook = _f32(codebook).reshape(self.M, self.ksub, self.d // self.M)
        self.cnorm = norms(self.centroids)
        self.T1 = precompute_T1(self.centroids, self.codebook)

    def train(self, x, niter_coarse=25, niter_pq=25, seed=1234):
        x = _f32(x)
        cent = np.empty((self.nlist, self.d), np.float32)
        cb = np.empty((self.M, self.ksub, self.d // self.M), np.float32)
        lib().or_train_ivfpq_metric(_p(x, _f32p), x.shape[0], self.d, self.nlist, self.M, self.ksub, niter_coarse,
                                    niter_pq, seed, _p(cent, _f32p), _p(cb, _f32p), self.nthreads, self.metric)
        self.set_trained(cent, cb)

    def encode(self, x):
        x = _f32(x)
        n = x.shape[0]
        lists = np.empty(n, np.int64)
        codes = np.empty((n, self.M), np.uint8)
        lib().or_encode_metric(_p(x, _f32p), n, self.d, _p(self.centroids, _f32p), _p(self.cnorm, _f32p),
                               self.nlist, _p(self.codebook, _f32p), self.M, self.ksub, _p(lists, _i64p),
                               _p(codes, _u8p), self.nthreads, self.metric)
        return lists, codes

    def add_preencoded(self, lists, codes, ids):
        order = np.argsort(lists, kind="stable")
        ls = lists[order]
        bounds = np.searchsorted(ls, np.arange(self.nlist + 1))
        for l in range(self.nlist):
            sel = order[bounds[l]:bounds[l + 1]]
            if sel.size:
                self.list_codes[l] = np.concatenate([self.list_codes[l], codes[sel]])
                self.list_ids[l] = np.concatenate([self.list_ids[l], ids[sel]])
        self.ntotal += lists.shape[0]

    def add_with_ids(self, x, ids):
        lists, codes = self.encode(x)
        self.add_preencoded(lists, codes, np.ascontiguousarray(ids, np.int64))

    def add(self, x):
        n = np.asarray(x).shape[0]
        self.add_with_ids(x, np.arange(self.ntotal, self.ntotal + n, dtype=np.int64))

    def invlists_flat(self):
        sizes = np.array([c.shape[0] for c in self.list_codes], np.int64)
        off = np.zeros(self.nlist + 1, np.int64)
        off[1:] = np.cumsum(sizes)
        codes = np.ascontiguousarray(np.concatenate(self.list_codes) if self.ntotal else
                                     np.zeros((0, self.M), np.uint8))
        ids = np.ascontiguousarray(np.concatenate(self.list_ids) if self.ntotal else np.zeros(0, np.int64))
        return off, codes, ids

    def search_preassigned(self, x, k, lists, dis0=None, nthreads=None):
        x = _f32(x)
        n = x.shape[0]
        lists = np.ascontiguousarray(lists, np.int64)
        nprobe = lists.shape[1]
        if dis0 is None:
            dis0 = np.zeros(lists.shape, np.float32)
        dis0 = _f32(dis0)
        off, codes, ids = self.invlists_flat()
        D = np.empty((n, k), np.float32)
        I = np.empty((n, k), np.int64)
        lib().or_search_preassigned_metric(_p(x, _f32p), n, self.d, _p(self.T1, _f32p), _p(self.codebook, _f32p),
                                           self.M, self.ksub, _p(off, _i64p), _p(codes, _u8p), _p(ids, _i64p),
                                           nprobe, _p(lists, _i64p), _p(dis0, _f32p), k, _p(D, _f32p),
                                           _p(I, _i64p), nthreads or self.nthreads, self.metric,
                                           _p(self.centroids, _f32p))
        return D, I

    def search(self, x, k, nthreads=None):
        dis, lists = coarse_search(x, self.centroids, self.nprobe, nthreads or self.nthreads, self.metric)
        return self.search_preassigned(x, k, lists, dis, nthreads)
