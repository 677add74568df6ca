"""CPU oracle pinning (no GPU): the oracle against the committed golden vectors,
the reference's own NumPy IVF-PQ search and the FPGA LUT known-answer test."""
import os

import numpy as np
import pytest

from oracle import oracle as O

CASES = ["d128_m16", "d64_m32_dsub2", "d96_m8_dsub12"]


def load(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name)))


def oracle_from(z):
    d, M, nlist = int(z["d"]), int(z["M"]), int(z["nlist"])
    ox = O.OracleIVFPQ(d, nlist, M)
    ox.set_trained(z["centroids"], z["codebook"])
    list_no = np.repeat(np.arange(nlist, dtype=np.int64), np.diff(z["list_off"]))
    ox.add_preencoded(list_no, z["codes"], z["ids"])
    ox.nprobe = int(z["nprobe"])
    return ox


@pytest.mark.parametrize("case", CASES)
def test_oracle_reproduces_golden_bit_exact(golden_dir, case):
    z = load(golden_dir, f"ivfpq_{case}.npz")
    ox = oracle_from(z)
    dis, lists = O.coarse_search(z["xq"], z["centroids"], int(z["nprobe"]))
    np.testing.assert_array_equal(lists, z["or_lists"])
    np.testing.assert_array_equal(dis, z["or_dis0"])
    D, I = ox.search(z["xq"], int(z["k"]))
    np.testing.assert_array_equal(I, z["or_I"])
    np.testing.assert_array_equal(D, z["or_D"])
    # thread count must not change results (queries are independent)
    D1, I1 = ox.search(z["xq"], int(z["k"]), nthreads=1)
    np.testing.assert_array_equal(I1, I)
    np.testing.assert_array_equal(D1, D)


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference_notebook(golden_dir, case):
    """IVFPQ_1B_search.ipynb cell 20 (run by tests/golden/make_golden.py) uses the
    residual LUT with float64 accumulation.  Distances agree within the
    north-star tolerance; labels agree except inside exact/near-tie groups,
    which the notebook orders by scan order and the oracle by label."""
    z = load(golden_dir, f"ivfpq_{case}.npz")
    D, I = z["or_D"].astype(np.float64), z["or_I"]
    nbD, nbI = z["nb_dists"], z["nb_ids"]
    np.testing.assert_allclose(D, nbD, rtol=1e-4)
    # a label the notebook puts in slot j instead of the oracle's must be a tie:
    # its own distance (the PQ reconstruction in float64, independent of both
    # codes' summation orders) equals the slot's distance
    M, d = int(z["M"]), int(z["d"])
    dsub = d // M
    pos_of = {int(v): i for i, v in enumerate(z["ids"])}
    list_of = np.repeat(np.arange(len(z["list_off"]) - 1), np.diff(z["list_off"]))
    cent, cb = z["centroids"].astype(np.float64), z["codebook"].astype(np.float64)

    def pq_dist(q, label):
        i = pos_of[int(label)]
        rec = cent[list_of[i]] + np.concatenate([cb[m, z["codes"][i, m]] for m in range(M)])
        return float(np.sum((z["xq"][q].astype(np.float64) - rec) ** 2))

    mism = 0
    for q in range(I.shape[0]):
        for j in np.where(I[q] != nbI[q])[0]:
            mism += 1
            tol = 1e-4 * max(1.0, abs(D[q, j]))
            assert abs(pq_dist(q, nbI[q, j]) - D[q, j]) <= tol, (case, q, j)
            assert abs(pq_dist(q, I[q, j]) - D[q, j]) <= tol, (case, q, j)
    assert mism <= 0.1 * I.size, (case, mism)  # ties are the exception, not the rule


@pytest.mark.parametrize("M", [32, 16])
def test_lut_known_answer(golden_dir, M):
    """FPGA LUT KAT (LUT_construction_PE_D128_M32/src/host.cpp:44-109): with
    integer inputs the Faiss table route T1 + (-2) T3 plus |r_m|^2 equals the
    residual LUT exactly."""
    z = load(golden_dir, "lut_kat.npz")
    q, c = z["query"], z["center"]
    cb = z[f"codebook_M{M}"]
    kat = z[f"lut_M{M}"]  # [256][M]
    T1 = O.precompute_T1(c[None, :], cb)[0]  # [M][256]
    T3 = O.ip_table(q[None, :], cb)[0]
    lut = T1 + (-2.0 * T3).astype(np.float32)
    r = (q - c).reshape(M, -1)
    rn = (r.astype(np.float64) ** 2).sum(1).astype(np.float32)
    np.testing.assert_array_equal(lut + rn[:, None], kat.T)


def test_tree_reduction_order():
    rng = np.random.default_rng(1)
    f = np.float32
    for d in (1, 2, 3, 4, 7, 8, 12, 16, 24):
        x = rng.standard_normal(d).astype(np.float32)
        y = rng.standard_normal(d).astype(np.float32)
        p = (x * y).astype(np.float32)
        a8 = np.zeros(8, np.float32)
        i = 0
        while i + 8 <= d:
            a8 = (a8 + p[i:i + 8]).astype(np.float32)
            i += 8
        a4 = (a8[4:] + a8[:4]).astype(np.float32)
        if i + 4 <= d:
            a4 = (a4 + p[i:i + 4]).astype(np.float32)
            i += 4
        for j in range(d - i):
            a4[j] = f(a4[j] + p[i + j])
        ref = f(f(a4[0] + a4[1]) + f(a4[2] + a4[3]))
        assert O.tree(x, y, 0) == ref, d


def test_kmeans_deterministic_and_train_encode():
    from faiss_amd import datasets

    x = datasets.synthetic_sift_like(3000, 16, seed=3, n_centres=20)
    c1 = O.kmeans(x, 16, 5, 7)
    c2 = O.kmeans(x, 16, 5, 7, nthreads=1)
    np.testing.assert_array_equal(c1, c2)
    ox = O.OracleIVFPQ(16, 8, 4)
    ox.train(x, niter_coarse=4, niter_pq=4, seed=5)
    lists, codes = ox.encode(x[:200])
    assert lists.min() >= 0 and lists.max() < 8
    assert codes.shape == (200, 4)
    ox.add(x)
    assert ox.ntotal == 3000
    ox.nprobe = 8
    D, I = ox.search(x[:10], 5)
    assert np.all(np.diff(D, axis=1) >= 0)


def test_preassigned_zero_coarse_default(golden_dir):
    z = load(golden_dir, "ivfpq_d128_m16.npz")
    ox = oracle_from(z)
    D0, I0 = ox.search_preassigned(z["xq"], 10, z["or_lists"], None)
    Dz, Iz = ox.search_preassigned(z["xq"], 10, z["or_lists"], np.zeros_like(z["or_dis0"]))
    np.testing.assert_array_equal(I0, Iz)
    np.testing.assert_array_equal(D0, Dz)
    D, I = ox.search_preassigned(z["xq"], 10, z["or_lists"], z["or_dis0"])
    np.testing.assert_array_equal(I, z["or_I"])


def test_padding_fewer_than_k():
    rng = np.random.default_rng(0)
    ox = O.OracleIVFPQ(16, 4, 4)
    ox.set_trained(rng.standard_normal((4, 16)), rng.standard_normal((4, 256, 4)))
    ox.add(rng.standard_normal((5, 16)).astype(np.float32))
    ox.nprobe = 4
    D, I = ox.search(rng.standard_normal((3, 16)).astype(np.float32), 8)
    assert np.all(I[:, 5:] == -1)
    assert np.all(D[:, 5:] == np.finfo(np.float32).max)


def test_oracle_inner_product_semantics():
    """METRIC_INNER_PRODUCT (beir/beir/retrieval/search/dense/faiss_search.py:170,
    194), checked against a direct restatement on integer-valued data (every
    product and sum is exact, so only the semantics are under test): coarse =
    the nprobe largest <q, c>; dis0 = <q, c_l>; LUT = T3; the k largest
    dis0 + sum_m T3[m][code_m], descending, ties by label; padding (-FLT_MAX, -1).
    Parity with Faiss itself is unpinned (the reference's oracle is L2-only)."""
    rng = np.random.default_rng(7)
    d, M, nlist, nprobe, k = 16, 4, 8, 3, 7
    cent = rng.integers(-3, 4, size=(nlist, d)).astype(np.float32)
    cb = rng.integers(-3, 4, size=(M, 256, d // M)).astype(np.float32)
    ox = O.OracleIVFPQ(d, nlist, M, metric=O.METRIC_INNER_PRODUCT)
    ox.set_trained(cent, cb)
    nb = 300
    lists = rng.integers(0, nlist, size=nb).astype(np.int64)
    lists[lists == 5] = 4  # list 5 stays empty
    codes = rng.integers(0, 256, size=(nb, M)).astype(np.uint8)
    codes[10:40] = codes[0]  # exact ties
    ids = rng.permutation(nb).astype(np.int64) * 3
    ox.add_preencoded(lists, codes, ids)
    ox.nprobe = nprobe
    xq = rng.integers(-3, 4, size=(6, d)).astype(np.float32)
    D, I = ox.search(xq, k)
    dsub = d // M
    for q in range(xq.shape[0]):
        x = xq[q].astype(np.float64)
        sims = cent.astype(np.float64) @ x
        probes = sorted(range(nlist), key=lambda l: (-sims[l], l))[:nprobe]
        t3 = np.einsum("mjt,mt->mj", cb.astype(np.float64), x.reshape(M, dsub))
        cand = []
        for l in probes:
            for i in np.where(lists == l)[0]:
                cand.append((sims[l] + sum(t3[m, codes[i, m]] for m in range(M)), ids[i]))
        cand.sort(key=lambda t: (-t[0], t[1]))
        cand = cand[:k]
        exp_I = [c[1] for c in cand] + [-1] * (k - len(cand))
        exp_D = [c[0] for c in cand] + [-np.finfo(np.float32).max] * (k - len(cand))
        np.testing.assert_array_equal(I[q], exp_I)
        np.testing.assert_array_equal(D[q], np.array(exp_D, np.float32))
    dis, lst = O.coarse_search(xq, cent, nprobe, metric=O.METRIC_INNER_PRODUCT)
    assert np.all(np.diff(dis, axis=1) <= 0)
    # preassigned: the coarse similarities passed in are not used (dis0 is recomputed)
    D2, I2 = ox.search_preassigned(xq, k, lst, np.zeros_like(dis))
    np.testing.assert_array_equal(I2, I)
    np.testing.assert_array_equal(D2, D)


def test_ip_kmeans_is_spherical_and_balanced():
    """Inner-product k-means is spherical, as Faiss's IndexIVF sets it for
    METRIC_INNER_PRODUCT (fvec_renorm_L2 after the initialization and after every
    update): unit-norm centroids, and on raw non-negative data no few large-norm
    centroids take almost every vector."""
    rng = np.random.default_rng(3)
    centres = rng.uniform(0, 128, (40, 32))
    x = np.clip(np.rint(centres[rng.integers(0, 40, 8000)] + rng.normal(0, 16, (8000, 32))), 0, 255).astype(np.float32)
    cent = O.kmeans(x, 32, 10, 5, nthreads=4, metric=O.METRIC_INNER_PRODUCT)
    np.testing.assert_allclose(np.linalg.norm(cent.astype(np.float64), axis=1), 1.0, rtol=1e-5)
    assign = np.argmax(x @ cent.T, axis=1)
    sizes = np.bincount(assign, minlength=32)
    assert sizes.max() < 0.25 * len(x), sizes
    assert (sizes > 0).sum() >= 24, sizes
