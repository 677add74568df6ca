"""The reference's GPU index key, "OPQ16,IVF262144,PQ16" at d = 128
(Chameleon/Faiss_experiments/bench_gpu_1bn.py:10, 17), searched on the GPU and
checked against the CPU oracle.

What this size exercises that smaller tests do not:
* the segmented coarse quantizer at nlist 262 144 (2 048 key tiles per query),
  both in the search and in the device add's top-1 assignment;
* a 4 GB precomputed table T1 (262 144 x 16 x 256 floats) built on the GPU;
* the per-list merge of the device add at nlist > 65 536 (the k_merge_lists grid
  cap of 65 535 lists per launch);
* tiny lists (about 2 codes each): many items per query, nearly all one code.

The index is not trained here (k-means over 262 144 centroids needs as many
training vectors and proves nothing about search parity): the OPQ rotation is a
random orthonormal matrix (what OPQMatrix.train also produces), the centroids
are 262 144 rotated synthetic vectors and the PQ codebook is 256 sampled
residuals per sub-space.  The oracle holds the same quantizers and the GPU's
lists; the queries are rotated by the oracle's own transform.
"""
import numpy as np
import pytest

import faiss_amd as faiss
from faiss_amd import datasets
from oracle import oracle as O

# (the module fixture builds a 4 GB table twice, on the GPU and in the oracle)
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

D_, NLIST, M = 128, 262_144, 16


@pytest.fixture(scope="module")
def opq_ivf262144():
    import torch

    rng = np.random.default_rng(5)
    q, r = np.linalg.qr(rng.standard_normal((D_, D_)))
    opq = faiss.OPQMatrix(D_, M)
    opq.set_matrix((q * np.sign(np.diag(r))[None, :]).T.astype(np.float32))
    xs = datasets.synthetic_sift_like(NLIST + 8192, D_, seed=31, n_centres=200_000)
    xs_t = O.linear_transform(xs, opq.A)
    cent = np.ascontiguousarray(xs_t[:NLIST])
    samp = np.ascontiguousarray(xs_t[NLIST:])
    ivf = faiss.IndexIVFPQ(None, D_, NLIST, M, 8, device=0)
    # codebook: 256 residuals of sample vectors to their nearest centroid, per sub-space
    ivf.set_trained(cent, np.zeros((M, 256, D_ // M), np.float32))
    ivf.nprobe = 1
    _, a = ivf.coarse_device(torch.from_numpy(samp).cuda())
    res = samp - cent[a[:, 0].cpu().numpy()]
    pick = rng.choice(res.shape[0], 256, replace=False)
    cb = np.ascontiguousarray(res[pick].reshape(256, M, D_ // M).transpose(1, 0, 2), np.float32)
    ivf.set_trained(cent, cb)
    ix = faiss.IndexPreTransform(opq, ivf)
    xb = datasets.synthetic_sift_like(600_000, D_, seed=32, n_centres=200_000)
    for i0 in range(0, xb.shape[0], 200_000):  # three device adds: pending entries merged per list
        ix.add(xb[i0:i0 + 200_000])
    xq = datasets.synthetic_sift_like(128, D_, seed=33, n_centres=200_000)
    ox = O.OracleIVFPQ(D_, NLIST, M)
    ox.set_trained(ivf.centroids(), ivf.codebook())
    lists, codes, ids = ivf.invlists.export()
    ox.add_preencoded(lists, codes, ids)
    return ix, ivf, ox, opq, xb, xq


def test_t1_and_lists(opq_ivf262144):
    """The 4 GB T1 equals the oracle's (rows of the first, a middle and the last
    lists), the lists hold every vector once, and a sample of the device add's
    assignments and codes equals the oracle's encode of the rotated vectors."""
    ix, ivf, ox, opq, xb, _ = opq_ivf262144
    assert ivf.ntotal == xb.shape[0]
    sizes = ivf.invlists.list_sizes()
    assert sizes.shape == (NLIST,) and int(sizes.sum()) == xb.shape[0]
    assert (sizes > 0).sum() > NLIST // 2  # lists past 65 536 are populated too
    assert sizes[200_000:].sum() > 0
    T1 = ivf.precomputed_table.reshape(NLIST, M, 256)
    for l in (0, 131_071, 200_000, NLIST - 1):
        np.testing.assert_array_equal(T1[l], ox.T1.reshape(NLIST, M, 256)[l])
    lists, codes, ids = ivf.invlists.export()
    sel = np.nonzero(ids < 600)[0]
    o = sel[np.argsort(ids[sel])]
    lo, co = ox.encode(O.linear_transform(xb[:600], opq.A))
    np.testing.assert_array_equal(lists[o], lo)
    np.testing.assert_array_equal(codes[o], co)


@pytest.mark.parametrize("nprobe,k", [(16, 10), (64, 100)])
def test_search_matches_oracle(opq_ivf262144, nprobe, k):
    ix, ivf, ox, opq, _, xq = opq_ivf262144
    ix.nprobe = ox.nprobe = nprobe
    D, I = ix.search(xq, k)
    Dr, Ir = ox.search(O.linear_transform(xq, opq.A), k)
    np.testing.assert_array_equal(I, Ir)
    np.testing.assert_array_equal(D, Dr)
    assert ivf.error_count() == 0 and ivf.repair_stats() == (0, 0)


def test_coarse_step_matches_oracle(opq_ivf262144):
    """The segmented coarse quantizer over 262 144 centroids (2 048 tiles of 128)."""
    import torch

    ix, ivf, ox, opq, _, xq = opq_ivf262144
    ix.nprobe = 32
    xt = O.linear_transform(xq, opq.A)
    Dq, Iq = ivf.coarse_device(torch.from_numpy(xt).cuda())
    Dr, Ir = O.coarse_search(xt, ivf.centroids(), 32)
    np.testing.assert_array_equal(Iq.cpu().numpy(), Ir)
    np.testing.assert_array_equal(Dq.cpu().numpy(), Dr)
