"""Caller replays: the reference's own call sequences for
this path, run call for call against faiss_amd, every search checked against the
oracle holding the same trained quantizers and lists.

* Chameleon/Faiss_experiments/IVFPQ_random_dataset.py:17-46 -- IndexFlatL2
  quantizer object, IndexIVFPQ(quantizer, d, 1024, 8, 8), uniform random data with
  the column-0 ramp, train, add, search(xb[:5]) at the default nprobe, nprobe = 16,
  then searches of 1, 10, ..., 10^4 queries (nb reduced from 1e6 to 200k so the
  oracle side stays fast; the calls are the script's).
* beir/beir/retrieval/search/dense/faiss_index.py:20-26, 80-96 (FaissTrainIndex.build
  + FaissIndex.search) with the IVF-PQ inner-product index of the C3 shape
  (faiss_search.py:170): train, adds in 50k chunks (FaissIndex.build's
  buffer_size), search(q, 1000), then the caller's ``_passage_ids[ids]`` lookup,
  which maps a -1 label to the last passage id; the -1 rows must be where the
  oracle has them, so the mapped ids agree too.
"""
import numpy as np
import pytest

import faiss_amd as faiss
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _oracle_like(ix, metric=O.METRIC_L2):
    ox = O.OracleIVFPQ(ix.d, ix.nlist, ix.M, metric=metric)
    ox.set_trained(ix.centroids(), ix.codebook())
    for l in range(ix.nlist):
        ox.list_ids[l] = ix.invlists.get_ids(l)
        ox.list_codes[l] = ix.invlists.get_codes(l).reshape(-1, ix.M)
    ox.ntotal = ix.ntotal
    return ox


def test_ivfpq_random_dataset_replay():
    d = 128
    nb = 200_000
    nq = int(1e4)
    np.random.seed(1234)
    xb = np.random.random((nb, d)).astype("float32")
    xb[:, 0] += np.arange(nb) / 1000.
    xq = np.random.random((nq, d)).astype("float32")
    xq[:, 0] += np.arange(nq) / 1000.

    nlist, nprob, m, nbits, topk = 1024, 16, 8, 8, 10
    quantizer = faiss.IndexFlatL2(d)
    index = faiss.IndexIVFPQ(quantizer, d, nlist, m, nbits)
    index.train(xb)
    index.add(xb)
    D, I = index.search(xb[:5], topk)  # sanity check, default nprobe (1)
    ox = _oracle_like(index)
    ox.nprobe = index.nprobe
    assert index.nprobe == 1
    Do, Io = ox.search(xb[:5], topk)
    np.testing.assert_array_equal(I, Io)
    np.testing.assert_array_equal(D, Do)
    assert quantizer.ntotal == nlist  # the quantizer object holds the trained centroids

    index.nprobe = nprob
    ox.nprobe = nprob
    for i in range(5):
        nq_range = int(10 ** i)
        D, I = index.search(xq[:nq_range], topk)
        Do, Io = ox.search(xq[:nq_range], topk)
        np.testing.assert_array_equal(I, Io, err_msg=f"nq_range={nq_range}")
        np.testing.assert_array_equal(D, Do, err_msg=f"nq_range={nq_range}")
    assert index.error_count() == 0


def test_beir_faiss_train_index_replay():
    rng = np.random.default_rng(5)
    d, n, nlist, M = 768, 120_000, 256, 64
    centres = rng.standard_normal((400, d)).astype(np.float32)
    emb = (centres[rng.integers(0, 400, n)] + 0.35 * rng.standard_normal((n, d))).astype(np.float32)
    emb /= np.linalg.norm(emb, axis=1, keepdims=True)
    queries = (emb[rng.integers(0, n, 48)] + 0.05 * rng.standard_normal((48, d))).astype(np.float32)
    passage_ids = np.array(rng.permutation(n) + 10_000, dtype=np.int64)  # FaissIndex(passage_ids)

    index = faiss.IndexIVFPQ(faiss.IndexFlatIP(d), d, nlist, M, 8, faiss.METRIC_INNER_PRODUCT)
    index.niter_coarse = index.niter_pq = 10
    # FaissTrainIndex.build: train on every embedding, then FaissIndex.build's 50k-chunk adds
    index.train(emb)
    buffer_size = 50000
    for start in range(0, len(passage_ids), buffer_size):
        index.add(emb[start:start + buffer_size])
    index.nprobe = 2  # few probes: k = 1000 outruns the candidates of some queries (-1 labels)
    k = 1000
    scores_arr, ids_arr = index.search(queries, k)
    mapped = passage_ids[ids_arr.reshape(-1)].reshape(queries.shape[0], -1)  # faiss_index.py:24-25

    ox = _oracle_like(index, O.METRIC_INNER_PRODUCT)
    ox.nprobe = 2
    Do, Io = ox.search(queries, k)
    np.testing.assert_array_equal(ids_arr, Io)
    np.testing.assert_array_equal(scores_arr, Do)
    assert (ids_arr == -1).any(), "the replay must exercise the -1 label case"
    np.testing.assert_array_equal(mapped, passage_ids[Io.reshape(-1)].reshape(queries.shape[0], -1))
    # the caller's silent mapping: -1 rows become the last passage id, with the Faiss
    # heap's neutral score (-FLT_MAX for inner product)
    assert (mapped[ids_arr == -1] == passage_ids[-1]).all()
    assert (scores_arr[ids_arr == -1] == -np.finfo(np.float32).max).all()
    assert index.error_count() == 0
