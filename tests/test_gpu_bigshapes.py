"""GPU parity at the two BASELINE.json shapes that need real list sizes, through
the C-ABI, bit-exact against the CPU oracle holding the same lists.

* C4 per-GPU shard (configs[3]: Deep1B-shaped, d 96, IVF65536,PQ48, nprobe 32,
  list-range sharded over 8 GPUs): rank 0's lists [0, 8192) filled with 16 M
  vectors generated on the device around those lists' centroids and added
  through add_device in 4 M slices (profiles/c4_shard.py builds the full 125 M
  shard the same way), so lists hold ~2 000 codes, not the ~6 of the reduced
  C4-shape test.  64 queries of the global distribution at k = 10 and 100.
  Reference flow: bench_gpu_1bn.py:598-658 (sharded add), :605-616 (shards).
* RALM retrieval shape (configs[4]'s retrieval stage): IVF32768,PQ32 at d 512,
  the reference's Dec-S config (Chameleon/llm_inference_gpu/experiments/config/
  Dec-S.yaml:15-19), served as FaissServer requests (ralm/server/
  faiss_server.py:170-239) of batch 32: the answer bytes must equal
  encode_answer of the oracle's search / search_preassigned.
"""
import numpy as np
import pytest

import faiss_amd as faiss
from faiss_amd import datasets, wire
from faiss_amd.server import RetrievalService
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def assert_same(D, I, Dr, Ir):
    np.testing.assert_array_equal(I, Ir)
    np.testing.assert_array_equal(D, Dr)


def oracle_lists(ix):
    ox = O.OracleIVFPQ(ix.d, ix.nlist, ix.M)
    ox.set_trained(ix.centroids(), ix.codebook())
    ox.add_preencoded(*ix.invlists.export())
    assert ox.ntotal == ix.ntotal
    return ox


@pytest.fixture(scope="module")
def c4_rank0_shard():
    import torch

    d, nlist, M, shards = 96, 65536, 48, 8
    xt = datasets.synthetic_sift_like(300_000, d, seed=4321 + 11, n_centres=200_000)
    ix = faiss.index_factory(d, f"IVF{nlist},PQ{M}", device=0)
    ix.niter_coarse = ix.niter_pq = 4
    ix.train(xt)
    lo, hi = 0, nlist // shards
    ix.set_list_range(lo, hi)
    dev = torch.device("cuda", 0)
    cent = torch.from_numpy(ix.centroids()[lo:hi]).to(dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    for _ in range(4):  # 4 x 4 M vectors, each slice one add_device
        n = 4_000_000
        which = torch.randint(0, hi - lo, (n,), device=dev, generator=g)
        x = torch.clamp(torch.round(cent[which] + 16.0 * torch.randn((n, d), device=dev, generator=g)), 0, 255)
        ix.add_device(x.contiguous())
        del x, which
    torch.cuda.synchronize()
    ix.nprobe = 32
    ox = oracle_lists(ix)
    ox.nprobe = 32
    xq = datasets.synthetic_sift_like(64, d, seed=123, n_centres=200_000)
    return ix, ox, xq, (lo, hi)


@pytest.mark.parametrize("k", [10, 100])
def test_c4_rank0_shard_16m_vectors(c4_rank0_shard, k):
    ix, ox, xq, (lo, hi) = c4_rank0_shard
    sizes = ix.invlists.list_sizes()
    assert ix.ntotal > 15_000_000  # the few vectors assigned outside [lo, hi) were dropped
    assert sizes[lo:hi].mean() > 1500 and sizes[hi:].sum() == 0
    D, I = ix.search(xq, k)
    Dr, Ir = ox.search(xq, k)
    assert_same(D, I, Dr, Ir)
    # a query's 32 probes miss the shard's eighth of the lists with probability ~ (7/8)^32
    assert (I[:, 0] >= 0).mean() > 0.9
    assert ix.error_count() == 0


@pytest.fixture(scope="module")
def ralm_dec_s():
    d, nlist, M = 512, 32768, 32
    xt = datasets.synthetic_sift_like(70_000, d, seed=11, n_centres=50_000)
    ix = faiss.index_factory(d, f"IVF{nlist},PQ{M}", device=0)
    ix.niter_coarse = ix.niter_pq = 4
    ix.train(xt)
    for i0 in range(0, 500_000, 250_000):
        ix.add(datasets.synthetic_sift_like(250_000, d, seed=100 + i0, n_centres=50_000))
    ix.nprobe = 32
    ox = oracle_lists(ix)
    ox.nprobe = 32
    xq = datasets.synthetic_sift_like(64, d, seed=7, n_centres=50_000)
    return ix, ox, xq


@pytest.mark.parametrize("k", [10, 100])
def test_ralm_dec_s_serve_request(ralm_dec_s, k):
    ix, ox, xq = ralm_dec_s
    b, dim = 32, xq.shape[1]
    q = np.ascontiguousarray(xq[:b])
    svc = RetrievalService(ix, batch_size=b, default_k=k, nprobe=32)
    ans = svc.handle(wire.encode_request(q, k, b, dim))
    Dr, Ir = ox.search(q, k)
    assert bytes(ans) == bytes(wire.encode_answer(Ir, Dr, k, b))


def test_ralm_dec_s_serve_request_with_lists(ralm_dec_s):
    # the IndexScanner path (ralm/index_scanner/index_scanner.py:61-77): the coarse
    # lists come from elsewhere with the request; search_preassigned without Dq
    ix, ox, xq = ralm_dec_s
    b, k, np_ = 32, 10, 32
    q = np.ascontiguousarray(xq[b:2 * b])
    _, lists = ix.quantizer.search(q, np_)
    lists = np.ascontiguousarray(lists, np.int64)
    svc = RetrievalService(ix, batch_size=b, default_k=k, nprobe=np_, request_with_lists=1)
    ans = svc.handle(wire.encode_request_with_lists(q, lists, b, q.shape[1], np_, k))
    Dr, Ir = ox.search_preassigned(q, k, lists)
    assert bytes(ans) == bytes(wire.encode_answer(Ir, Dr, k, b))
    assert ix.error_count() == 0
