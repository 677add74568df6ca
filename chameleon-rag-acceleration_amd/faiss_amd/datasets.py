"""Dataset I/O, recall metrics and the synthetic SIFT1M-shaped generator.

Readers follow the reference's formats
(``Chameleon/Faiss_experiments/datasets.py:13-37`` for ``.fvecs/.ivecs``,
``:107-142`` for Deep ``.fbin/.ibin``; ``.bvecs`` as in ``mmap_bvecs``).
``evaluate`` reproduces the reference's R1@k definition
(``datasets.py:40-52``, ``bench_polysemous_1bn.py:432-434``): the fraction of
queries whose true nearest neighbour appears in the first k results.
``recall_at_k`` is the intersection recall R@k of
``bench_cpu_performance_OSDI.py:355-359``.

Nothing here touches the GPU.
"""
from __future__ import annotations

import time

import numpy as np


# The .ivecs/.fvecs readers and `evaluate` below follow the Faiss benchmark
# helpers (MIT licence) that the reference reuses in
# Chameleon/Faiss_experiments/datasets.py:13-52; the recall definition is kept
# identical on purpose so the bench's recall column means the same thing.
def ivecs_read(fname):
    a = np.fromfile(fname, dtype="int32")
    d = a[0]
    return a.reshape(-1, d + 1)[:, 1:].copy()


def fvecs_read(fname):
    return ivecs_read(fname).view("float32")


def ivecs_write(fname, m):
    m = np.ascontiguousarray(m, dtype=np.int32)
    n, d = m.shape
    out = np.empty((n, d + 1), np.int32)
    out[:, 0] = d
    out[:, 1:] = m
    out.tofile(fname)


def fvecs_write(fname, m):
    ivecs_write(fname, np.ascontiguousarray(m, dtype=np.float32).view("int32"))


def mmap_bvecs(fname):
    x = np.memmap(fname, dtype="uint8", mode="r")
    d = x[:4].view("int32")[0]
    return x.reshape(-1, d + 4)[:, 4:]


def mmap_fbin(fname):
    """Deep1B .fbin: int32 n, int32 d, then n*d float32."""
    hdr = np.fromfile(fname, dtype="int32", count=2)
    n, d = int(hdr[0]), int(hdr[1])
    return np.memmap(fname, dtype="float32", mode="r", offset=8, shape=(n, d))


def read_ibin(fname):
    hdr = np.fromfile(fname, dtype="int32", count=2)
    n, d = int(hdr[0]), int(hdr[1])
    return np.fromfile(fname, dtype="int32", offset=8).reshape(n, d)


def load_sift1M(root="sift1M"):
    xt = fvecs_read(f"{root}/sift_learn.fvecs")
    xb = fvecs_read(f"{root}/sift_base.fvecs")
    xq = fvecs_read(f"{root}/sift_query.fvecs")
    gt = ivecs_read(f"{root}/sift_groundtruth.ivecs")
    return xb, xq, xt, gt


def recall_1_at(I, gt, ranks=(1, 10, 100)):
    """R1@r: fraction of queries whose gt[:, 0] is within the first r labels."""
    I = np.asarray(I)
    gt = np.asarray(gt)
    nq = I.shape[0]
    out = {}
    for r in ranks:
        if r <= I.shape[1]:
            out[r] = float((I[:, :r] == gt[:, :1]).sum()) / nq
    return out


def recall_at_k(I, gt, k):
    """Intersection recall R@k = |top-k ∩ gt top-k| / k, averaged over queries."""
    I = np.asarray(I)[:, :k]
    gt = np.asarray(gt)[:, :k]
    hits = sum(len(np.intersect1d(I[i], gt[i])) for i in range(I.shape[0]))
    return hits / float(I.shape[0] * k)


def evaluate(index, xq, gt, k):
    nq = xq.shape[0]
    t0 = time.time()
    D, I = index.search(xq, k)
    t1 = time.time()
    recalls = {}
    i = 1
    while i <= k:
        recalls[i] = (I[:, :i] == gt[:, :1]).sum() / float(nq)
        i *= 10
    return (t1 - t0) * 1000.0 / nq, recalls


def synthetic_sift_like(n, d=128, seed=1234, n_centres=200_000, sigma=16.0, centre_seed=20251015):
    """Clustered, SIFT-like (non-negative integer valued) float32 vectors.

    SURVEY.md §8(d): Gaussian centres ~ U[0,128)^d shared by base, train and
    query sets; points = clip(round(centre + N(0, sigma^2)), 0, 255).  Uniform
    random data gives poor PQ recall (``Chameleon/Faiss_experiments/
    generate_SYN_dataset.py:4-5``).  The centre count is tuned so that the
    IVF1024,PQ16 recall-vs-nprobe curve tracks real SIFT1M's
    (``Chameleon/Faiss_experiments/README.md:266-273``: R1@10 0.8907 at nprobe
    16): 200,000 centres give 0.897 (10,000, the survey's first suggestion,
    saturate at 0.455: with ~100 points per tight blob the nearest neighbour is
    not separable by the PQ distances).  DESIGN.md §6 has both curves.
    """
    crng = np.random.default_rng(centre_seed)
    centres = crng.uniform(0.0, 128.0, size=(n_centres, d)).astype(np.float32)
    rng = np.random.default_rng(seed)
    out = np.empty((n, d), np.float32)
    bs = 1 << 16
    for i0 in range(0, n, bs):
        m = min(bs, n - i0)
        which = rng.integers(0, n_centres, size=m)
        pts = centres[which] + rng.normal(0.0, sigma, size=(m, d)).astype(np.float32)
        np.clip(np.rint(pts), 0, 255, out=pts)
        out[i0:i0 + m] = pts
    return out


def embed_like(x, mu):
    """Centred, unit-norm rows (sentence-embedding-like, the C3 shape): the raw
    non-negative synthetic rows have one dominant direction, which inner-product
    search would rank by norm alone."""
    y = x - mu
    return np.ascontiguousarray(y / np.maximum(np.linalg.norm(y, axis=1, keepdims=True), 1e-6), np.float32)


def c3_nq_shaped(nb=2_680_000, nt=200_000, nq=4096, d=768, n_centres=20000, seed0=7, chunk=500_000):
    """The C3 (BEIR-NQ-shaped) synthetic set: 768-d embedding-like rows
    (embed_like of synthetic_sift_like, centred on the training mean).
    Returns (xt, base chunk generator, xq); the base set is yielded in chunks of
    `chunk` rows (seeds 1000 + seed0 + i0), so 2.68 M x 768 floats never sit in
    host memory at once."""
    xt = synthetic_sift_like(nt, d, seed=4321 + seed0, n_centres=n_centres)
    mu = xt.mean(0, keepdims=True)
    xq = embed_like(synthetic_sift_like(nq, d, seed=123, n_centres=n_centres), mu)

    def base():
        for i0 in range(0, nb, chunk):
            yield embed_like(synthetic_sift_like(min(chunk, nb - i0), d, seed=1000 + seed0 + i0,
                                                 n_centres=n_centres), mu)

    return embed_like(xt, mu), base, xq


def sift1m_shaped(nb=1_000_000, nt=100_000, nq=10_240, d=128):
    """The C2 synthetic workload: base seed 1234, train 4321, queries 123."""
    xb = synthetic_sift_like(nb, d, seed=1234)
    xt = synthetic_sift_like(nt, d, seed=4321)
    xq = synthetic_sift_like(nq, d, seed=123)
    return xb, xt, xq


def brute_force_gt(xb, xq, k, block=4096):
    """Exact float64 k-NN (L2) on the host; for small sets (tests)."""
    xb64 = np.asarray(xb, np.float64)
    nb2 = (xb64 ** 2).sum(1)
    out = np.empty((xq.shape[0], k), np.int64)
    for i0 in range(0, xq.shape[0], block):
        q = np.asarray(xq[i0:i0 + block], np.float64)
        dd = (q ** 2).sum(1)[:, None] + nb2[None, :] - 2 * q @ xb64.T
        idx = np.argpartition(dd, kth=min(k, dd.shape[1] - 1), axis=1)[:, :k]
        part = np.take_along_axis(dd, idx, 1)
        o = np.lexsort((idx, part), axis=1)
        out[i0:i0 + block] = np.take_along_axis(idx, o, 1)
    return out
