"""METRIC_INNER_PRODUCT on the GPU against the oracle's IP restatement
(beir's default metric,
beir/beir/retrieval/search/dense/faiss_search.py:170, 194, with
EvaluateRetrieval's top_k = 1000, beir/beir/retrieval/evaluation.py:13, 20).

Bit-exact ids and similarities.  Parity unpinned beyond the oracle: the
reference's own NumPy oracle and the FPGA are L2-only, and Faiss is not
importable here (tests/test_oracle.py::test_oracle_inner_product_semantics pins
the oracle's IP semantics on exact integer data).
"""
import os

import numpy as np
import pytest

import faiss_amd as faiss
from faiss_amd import datasets
from faiss_amd.sharding import balanced_list_ranges
from oracle import oracle as O

pytestmark = pytest.mark.gpu
IP = faiss.METRIC_INNER_PRODUCT
CASES = ["d128_m16", "d64_m32_dsub2", "d96_m8_dsub12"]


def assert_same(D, I, Dr, Ir):
    np.testing.assert_array_equal(I, Ir)
    np.testing.assert_allclose(D, Dr, rtol=1e-4, atol=0)
    np.testing.assert_array_equal(D, Dr)


def pair_from_golden(golden_dir, case):
    z = dict(np.load(os.path.join(golden_dir, f"ivfpq_{case}.npz")))
    d, M, nlist = int(z["d"]), int(z["M"]), int(z["nlist"])
    list_no = np.repeat(np.arange(nlist, dtype=np.int64), np.diff(z["list_off"]))
    ix = faiss.IndexIVFPQ(None, d, nlist, M, 8, IP, device=0)
    ix.set_trained(z["centroids"], z["codebook"])
    ix.add_preencoded(list_no, z["codes"], z["ids"])
    ox = O.OracleIVFPQ(d, nlist, M, metric=O.METRIC_INNER_PRODUCT)
    ox.set_trained(z["centroids"], z["codebook"])
    ox.add_preencoded(list_no, z["codes"], z["ids"])
    ix.nprobe = ox.nprobe = int(z["nprobe"])
    # centre the queries so that similarities take both signs
    xq = z["xq"] - z["xq"].mean(0, keepdims=True)
    return ix, ox, np.ascontiguousarray(xq, np.float32), z


@pytest.mark.parametrize("case", CASES)
def test_ip_golden_indexes(golden_dir, case):
    ix, ox, xq, z = pair_from_golden(golden_dir, case)
    assert isinstance(ix.quantizer, faiss.IndexFlatIP)
    for k in (int(z["k"]), 100):
        D, I = ix.search(xq, k)
        Dr, Ir = ox.search(xq, k)
        assert_same(D, I, Dr, Ir)
        assert np.all(np.diff(D, axis=1) <= 0)


def test_ip_coarse_and_preassigned(golden_dir):
    import torch

    ix, ox, xq, z = pair_from_golden(golden_dir, "d128_m16")
    dis, lists = O.coarse_search(xq, z["centroids"], ix.nprobe, metric=O.METRIC_INNER_PRODUCT)
    Dq, Iq = ix.coarse_device(torch.from_numpy(xq).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(Iq.cpu().numpy(), lists)
    np.testing.assert_array_equal(Dq.cpu().numpy(), dis)
    # the coarse similarities handed in are not used (Faiss recomputes dis0 = <q, c>)
    D, I = ix.search_preassigned(xq, 10, lists, np.zeros_like(dis))
    Dr, Ir = ox.search_preassigned(xq, 10, lists)
    assert_same(D, I, Dr, Ir)
    lists[:, 1::3] = -1
    D, I = ix.search_preassigned(xq, 10, lists)
    Dr, Ir = ox.search_preassigned(xq, 10, lists)
    assert_same(D, I, Dr, Ir)


def test_ip_padding_and_flat():
    rng = np.random.default_rng(4)
    d, M, nlist = 32, 8, 16
    cent = rng.normal(size=(nlist, d)).astype(np.float32)
    cb = rng.normal(size=(M, 256, d // M)).astype(np.float32)
    ix = faiss.IndexIVFPQ(None, d, nlist, M, 8, IP, device=0)
    ix.set_trained(cent, cb)
    ox = O.OracleIVFPQ(d, nlist, M, metric=O.METRIC_INNER_PRODUCT)
    ox.set_trained(cent, cb)
    x = rng.normal(size=(40, d)).astype(np.float32)
    ix.add(x)
    ox.add_preencoded(*ox.encode(x), np.arange(40, dtype=np.int64))
    ix.nprobe = ox.nprobe = 2
    q = rng.normal(size=(9, d)).astype(np.float32)
    D, I = ix.search(q, 30)
    Dr, Ir = ox.search(q, 30)
    assert_same(D, I, Dr, Ir)
    assert (I == -1).any() and np.all(D[I == -1] == -np.finfo(np.float32).max)
    # IndexFlatIP: exact k largest inner products (integer data: exact)
    xb = rng.integers(-5, 6, size=(2000, 24)).astype(np.float32)
    xq = rng.integers(-5, 6, size=(20, 24)).astype(np.float32)
    fl = faiss.IndexFlatIP(24, device=0)
    fl.add(xb)
    D, I = fl.search(xq, 15)
    s = xq.astype(np.float64) @ xb.T.astype(np.float64)
    for r in range(xq.shape[0]):
        o = np.lexsort((np.arange(xb.shape[0]), -s[r]))[:15]
        np.testing.assert_array_equal(I[r], o)
        np.testing.assert_array_equal(D[r], s[r][o].astype(np.float32))


@pytest.fixture(scope="module")
def c3_ip():
    # BEIR-NQ-shaped, inner product: d = 768, M = 64, nb reduced to 60k
    xt = datasets.synthetic_sift_like(20_000, 768, seed=4321, n_centres=2000)
    xb = datasets.synthetic_sift_like(60_000, 768, seed=1234, n_centres=2000)
    xq = datasets.synthetic_sift_like(64, 768, seed=123, n_centres=2000)
    mu = xt.mean(0, keepdims=True)
    xt, xb, xq = (np.ascontiguousarray(a - mu, np.float32) for a in (xt, xb, xq))
    ix = faiss.index_factory(768, "IVF256,PQ64", IP)
    ix.niter_coarse = ix.niter_pq = 4
    ix.train(xt)
    ix.add(xb)
    ox = O.OracleIVFPQ(768, 256, 64, metric=O.METRIC_INNER_PRODUCT)
    ox.set_trained(ix.centroids(), ix.codebook())
    for l in range(256):
        ox.list_ids[l] = ix.invlists.get_ids(l)
        ox.list_codes[l] = ix.invlists.get_codes(l).reshape(-1, 64)
    ox.ntotal = ix.ntotal
    return ix, ox, xq


@pytest.mark.parametrize("k", [10, 1000])
def test_ip_c3_shape_k(c3_ip, k):
    """C3: 768-d, M = 64, nprobe = 32, IP, k up to beir's 1000."""
    ix, ox, xq = c3_ip
    ix.nprobe = ox.nprobe = 32
    D, I = ix.search(xq, k)
    Dr, Ir = ox.search(xq, k)
    assert_same(D, I, Dr, Ir)


def test_ip_nprobe_above_64(c3_ip):
    """nprobe > 64: the coarse kernel's multi-row selection, planned by k_plan_count."""
    ix, ox, xq = c3_ip
    ix.nprobe = ox.nprobe = 100
    D, I = ix.search(xq, 20)
    Dr, Ir = ox.search(xq, 20)
    assert_same(D, I, Dr, Ir)


def test_ip_shards_merge(c3_ip):
    import torch

    ix, ox, xq = c3_ip
    ix.nprobe = ox.nprobe = 32
    sizes = ix.invlists.list_sizes()
    xd = torch.from_numpy(xq).cuda()
    Ds, Is = [], []
    for lo, hi in balanced_list_ranges(sizes, 3, ix.M):
        sh = faiss.IndexIVFPQ(None, 768, 256, 64, 8, IP, device=0)
        sh.set_trained(ix.centroids(), ix.codebook())
        sh.set_list_range(lo, hi)
        ls = [l for l in range(lo, hi) if sizes[l]]
        sh.add_preencoded(np.concatenate([np.full(sizes[l], l, np.int64) for l in ls]),
                          np.concatenate([ix.invlists.get_codes(l).reshape(-1, 64) for l in ls]),
                          np.concatenate([ix.invlists.get_ids(l) for l in ls]))
        sh.nprobe = 32
        D, I = sh.search_device(xd, 50)
        Ds.append(D)
        Is.append(I)
    D, I = faiss.merge_topk_device(torch.stack(Ds), torch.stack(Is), metric=IP)
    torch.cuda.synchronize()
    Dr, Ir = ox.search(xq, 50)
    assert_same(D.cpu().numpy(), I.cpu().numpy(), Dr, Ir)


def test_ip_large_nlist_split_coarse():
    """nlist >= 8192 (not a multiple of the 128-centroid tile): the segmented coarse quantizer."""
    xt = datasets.synthetic_sift_like(12_000, 32, seed=4321, n_centres=5000)
    xb = datasets.synthetic_sift_like(60_000, 32, seed=1234, n_centres=5000)
    xq = datasets.synthetic_sift_like(40, 32, seed=123, n_centres=5000)
    mu = xt.mean(0, keepdims=True)
    xt, xb, xq = (np.ascontiguousarray(a - mu, np.float32) for a in (xt, xb, xq))
    ix = faiss.index_factory(32, "IVF9000,PQ8", IP)
    ix.niter_coarse = ix.niter_pq = 2
    ix.train(xt)
    ix.add(xb)
    ox = O.OracleIVFPQ(32, 9000, 8, metric=O.METRIC_INNER_PRODUCT)
    ox.set_trained(ix.centroids(), ix.codebook())
    for l in range(9000):
        ox.list_ids[l] = ix.invlists.get_ids(l)
        ox.list_codes[l] = ix.invlists.get_codes(l).reshape(-1, 8)
    ox.ntotal = ix.ntotal
    ix.nprobe = ox.nprobe = 24
    D, I = ix.search(xq, 10)
    Dr, Ir = ox.search(xq, 10)
    assert_same(D, I, Dr, Ir)


def test_ip_train_and_add_match_oracle():
    """IP index training (coarse k-means assigning by the largest inner product,
    residuals to that centroid, L2 PQ k-means) and add (IP assignment) equal the
    oracle's."""
    x = datasets.synthetic_sift_like(6000, 32, seed=7, n_centres=50)
    x = np.ascontiguousarray(x - x.mean(0, keepdims=True), np.float32)
    ix = faiss.IndexIVFPQ(None, 32, 16, 8, 8, IP, device=0)
    ix.niter_coarse, ix.niter_pq, ix.seed = 6, 5, 99
    ix.train(x)
    ox = O.OracleIVFPQ(32, 16, 8, metric=O.METRIC_INNER_PRODUCT)
    ox.train(x, niter_coarse=6, niter_pq=5, seed=99)
    np.testing.assert_array_equal(ix.centroids(), ox.centroids)
    np.testing.assert_array_equal(ix.codebook(), ox.codebook)
    ix.add(x[:3000])
    ox.add(x[:3000])
    for l in range(16):
        np.testing.assert_array_equal(ix.invlists.get_ids(l), ox.list_ids[l])
        np.testing.assert_array_equal(ix.invlists.get_codes(l).reshape(-1, 8), ox.list_codes[l])
    ix.nprobe = ox.nprobe = 4
    D, I = ix.search(x[3000:3100], 10)
    Dr, Ir = ox.search(x[3000:3100], 10)
    assert_same(D, I, Dr, Ir)


@pytest.mark.gpu
def test_ip_train_spherical_on_raw_data_matches_oracle():
    """IP training on raw non-negative rows (no centring): the GPU k-means is
    spherical like Faiss's (unit-norm centroids), equal to the oracle's bit for
    bit, and the lists stay balanced."""
    x = datasets.synthetic_sift_like(8000, 32, seed=11, n_centres=40)
    ix = faiss.IndexIVFPQ(None, 32, 32, 8, 8, IP, device=0)
    ix.niter_coarse, ix.niter_pq, ix.seed = 8, 4, 5
    ix.train(x)
    ox = O.OracleIVFPQ(32, 32, 8, metric=O.METRIC_INNER_PRODUCT)
    ox.train(x, niter_coarse=8, niter_pq=4, seed=5)
    np.testing.assert_array_equal(ix.centroids(), ox.centroids)
    np.testing.assert_array_equal(ix.codebook(), ox.codebook)
    np.testing.assert_allclose(np.linalg.norm(ix.centroids().astype(np.float64), axis=1), 1.0, rtol=1e-5)
    ix.add(x)
    sizes = ix.invlists.list_sizes()
    assert sizes.max() < 0.25 * len(x), sizes
