"""GPU: the OPQ / LinearTransform apply kernel (k_linear_transform through
ivfpq_linear_transform_device) and an "OPQ..,IVF..,PQ.." index end to end,
against the CPU oracle.

The apply follows or_linear_transform's t-ordered fmaf chain, so outputs are
bit-identical; the OPQ index is then an IVF-PQ over transformed vectors and its
search must equal the oracle's IVF-PQ (same trained quantizers, same codes) on
oracle-transformed queries, IDs and distances bit for bit.  OPQ training itself
is host numpy (test_transform.py) and not Faiss-pinned."""
import numpy as np
import pytest

import faiss_amd as faiss
from faiss_amd import datasets
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,d_in,d_out,bias", [(1000, 128, 128, False), (333, 96, 64, True), (1, 7, 3, False),
                                               (0, 16, 16, False)])
def test_apply_bit_exact(n, d_in, d_out, bias):
    import torch

    rng = np.random.default_rng(n + d_in)
    x = rng.standard_normal((n, d_in)).astype(np.float32) * 10
    lt = faiss.LinearTransform(d_in, d_out, bias)
    lt.set_matrix(rng.standard_normal((d_out, d_in)), rng.standard_normal(d_out) if bias else None)
    y = lt.apply(x)
    assert y.shape == (n, d_out)
    np.testing.assert_array_equal(y, O.linear_transform(x, lt.A, lt.b))
    with pytest.raises(RuntimeError):
        lt.apply_device(torch.zeros((4, d_in + 1), device="cuda"))


def test_opq_index_matches_oracle(tmp_path):
    import torch

    d = 64
    xt = datasets.synthetic_sift_like(6000, d, seed=11, n_centres=300)
    xb = datasets.synthetic_sift_like(20000, d, seed=12, n_centres=300)
    xq = datasets.synthetic_sift_like(200, d, seed=13, n_centres=300)
    ix = faiss.index_factory(d, "OPQ8,IVF64,PQ8")
    assert isinstance(ix, faiss.IndexPreTransform) and isinstance(ix.chain.at(0), faiss.OPQMatrix)
    ix.chain[0].niter = 4
    ix.train(xt)
    ix.add(xb)
    ix.nprobe = 8
    k = 10
    D, I = ix.search(xq, k)

    A = ix.chain.at(0).A
    ivf = faiss.downcast_index(ix.index)
    ox = O.OracleIVFPQ(d, 64, 8)
    ox.set_trained(ivf.centroids(), ivf.codebook())
    lists = np.concatenate([np.full(ivf.invlists.list_size(l), l, np.int64) for l in range(64)])
    codes = np.concatenate([ivf.invlists.get_codes(l).reshape(-1, 8) for l in range(64)])
    ids = np.concatenate([ivf.invlists.get_ids(l) for l in range(64)])
    ox.add_preencoded(lists, codes, ids)
    ox.nprobe = 8
    Dr, Ir = ox.search(O.linear_transform(xq, A), k)
    np.testing.assert_array_equal(I, Ir)
    np.testing.assert_array_equal(D, Dr)
    # the stored codes are the encoding of the oracle-transformed base vectors
    ob = O.OracleIVFPQ(d, 64, 8)
    ob.set_trained(ivf.centroids(), ivf.codebook())
    ob.add(O.linear_transform(xb, A))
    off_r, codes_r, ids_r = ob.invlists_flat()
    np.testing.assert_array_equal(np.diff(off_r), ivf.invlists.list_sizes())
    np.testing.assert_array_equal(ids_r, ids)
    np.testing.assert_array_equal(codes_r, codes)

    # device search path and Faiss-file round trip
    Dd, Id = ix.search_device(torch.from_numpy(xq).cuda(), k)
    np.testing.assert_array_equal(Id.cpu().numpy(), I)
    p = tmp_path / "opq.index"
    faiss.write_index(ix, str(p))
    back = faiss.read_index(str(p))
    assert isinstance(back, faiss.IndexPreTransform)
    np.testing.assert_array_equal(back.chain.at(0).A, A)
    back.nprobe = 8
    D2, I2 = back.search(xq, k)
    np.testing.assert_array_equal(I2, I)
    np.testing.assert_array_equal(D2, D)


def test_opq_index_full_surface():
    """An "OPQ..,IVF..,PQ.." index behind the rest of the surface: preassigned
    search (both forms), the coarse step on the device, a wire request through
    RetrievalService (plain and with lists) -- each equal to transforming the
    queries by hand and asking the wrapped IVF-PQ -- and the apply on a side
    stream equal to the apply on the current stream."""
    import torch

    from faiss_amd import wire
    from faiss_amd.server import RetrievalService

    d = 32
    xt = datasets.synthetic_sift_like(4000, d, seed=21, n_centres=100)
    xb = datasets.synthetic_sift_like(8000, d, seed=22, n_centres=100)
    xq = datasets.synthetic_sift_like(16, d, seed=23, n_centres=100)
    ix = faiss.index_factory(d, "OPQ8,IVF32,PQ8")
    ix.chain[0].niter = 2
    ix.train(xt)
    ix.add(xb)
    ix.nprobe = 4
    ivf = faiss.downcast_index(ix.index)
    xqt = ix.apply_chain(xq)
    k = 5
    Dref, Iref = ivf.search(xqt, k)
    D, I = ix.search(xq, k)
    np.testing.assert_array_equal(I, Iref)
    Iq = torch.empty((16, 4), dtype=torch.int64, device="cuda")
    Dq = torch.empty((16, 4), dtype=torch.float32, device="cuda")
    ix.coarse_device(torch.from_numpy(xq).cuda(), Iq, Dq)
    Dq2, Iq2 = ivf.coarse_device(torch.from_numpy(xqt).cuda())
    np.testing.assert_array_equal(Iq.cpu().numpy(), Iq2.cpu().numpy())
    lists = Iq.cpu().numpy()
    Dp, Ip = ix.search_preassigned(xq, k, lists)
    Dpr, Ipr = ivf.search_preassigned(xqt, k, lists)
    np.testing.assert_array_equal(Ip, Ipr)
    Dc, Ic = np.zeros((16, k), np.float32), np.zeros((16, k), np.int64)
    ix.search_preassigned(16, xq, k, lists, None, Dc, Ic, False)
    np.testing.assert_array_equal(Ic, Ipr)
    svc = RetrievalService(ix, batch_size=16, default_k=k, nprobe=4)
    ans = svc.handle(wire.encode_request(xq, k, 16, d))
    Ia, Da = wire.decode_answer(bytes(ans), k, 16)
    np.testing.assert_array_equal(Ia, Iref)
    np.testing.assert_array_equal(Da, Dref)
    svl = RetrievalService(ix, batch_size=16, default_k=k, nprobe=4, request_with_lists=1)
    ans = svl.handle(wire.encode_request_with_lists(xq, lists, 16, d, 4, k))
    Ia, Da = wire.decode_answer(bytes(ans), k, 16)
    np.testing.assert_array_equal(Ia, Ipr)
    # apply on a side stream (the output allocated on that stream, ordered after the current one)
    side = torch.cuda.Stream()
    xd = torch.from_numpy(xq).cuda()
    y = ix.chain.at(0).apply_device(xd, side.cuda_stream)
    side.synchronize()
    np.testing.assert_array_equal(y.cpu().numpy(), xqt)
