"""Full-size parity at C3 (BASELINE.json configs[2]): the 2.68 M-vector
IVF4096,PQ64 inner-product index over 768-d embedding-shaped rows that
profiles/config_rates.py times (datasets.c3_nq_shaped, GPU-trained), searched
at nprobe 32 with k = 10 and beir's top_k = 1000
(beir/beir/retrieval/evaluation.py:13, 20; faiss_search.py:170 for the
metric), bit-exact against the oracle holding the same trained index.
"""
import numpy as np
import pytest

import faiss_amd as faiss
from faiss_amd import datasets
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c3_full():
    xt, base, xq = datasets.c3_nq_shaped()
    ix = faiss.index_factory(768, "IVF4096,PQ64", faiss.METRIC_INNER_PRODUCT)
    ix.niter_coarse = ix.niter_pq = 6
    ix.train(xt)
    for xb in base():
        ix.add(xb)
    assert ix.ntotal == 2_680_000
    ox = O.OracleIVFPQ(768, 4096, 64, metric=O.METRIC_INNER_PRODUCT)
    ox.set_trained(ix.centroids(), ix.codebook())
    for l in range(4096):
        ox.list_ids[l] = ix.invlists.get_ids(l)
        ox.list_codes[l] = ix.invlists.get_codes(l).reshape(-1, 64)
    ox.ntotal = ix.ntotal
    return ix, ox, xq[:128]


@pytest.mark.parametrize("k", [10, 1000])
def test_c3_full_size_ip(c3_full, k):
    ix, ox, xq = c3_full
    ix.nprobe = ox.nprobe = 32
    D, I = ix.search(xq, k)
    Dr, Ir = ox.search(xq, k)
    np.testing.assert_array_equal(I, Ir)
    np.testing.assert_allclose(D, Dr, rtol=1e-4, atol=0)
    np.testing.assert_array_equal(D, Dr)
    assert np.all(np.diff(D, axis=1) <= 0)
    # every query has k results (the probed lists hold far more than 1000 vectors)
    assert (I >= 0).all()
