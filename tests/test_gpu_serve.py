"""FaissServer request handling on the GPU: one RALM wire
message in, the answer message out, through ``ivfpq_serve_request``.

Parity: the answer bytes must equal ``encode_answer`` (byte layout pinned by
tests/test_wire.py against the reference's encoder) of the oracle's search /
search_preassigned on the same golden index -- bit-exact ids and distances.
"""
import os

import numpy as np
import pytest

import faiss_amd as faiss
from faiss_amd import wire
from faiss_amd.server import RetrievalService
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def golden_pair(golden_dir, case="d128_m16"):
    z = dict(np.load(os.path.join(golden_dir, f"ivfpq_{case}.npz")))
    d, M, nlist = int(z["d"]), int(z["M"]), int(z["nlist"])
    list_no = np.repeat(np.arange(nlist, dtype=np.int64), np.diff(z["list_off"]))
    ix = faiss.IndexIVFPQ(None, d, nlist, M, 8, device=0)
    ix.set_trained(z["centroids"], z["codebook"])
    ix.add_preencoded(list_no, z["codes"], z["ids"])
    ox = O.OracleIVFPQ(d, nlist, M)
    ox.set_trained(z["centroids"], z["codebook"])
    ox.add_preencoded(list_no, z["codes"], z["ids"])
    ix.nprobe = ox.nprobe = int(z["nprobe"])
    return ix, ox, z


@pytest.mark.parametrize("k", [10, 100])
def test_serve_plain_request_matches_oracle(golden_dir, k):
    ix, ox, z = golden_pair(golden_dir)
    xq = np.ascontiguousarray(z["xq"][:32], np.float32)
    b, dim = xq.shape
    svc = RetrievalService(ix, batch_size=b, default_k=k, nprobe=ix.nprobe)
    msg = wire.encode_request(xq, k, b, dim)
    ans = svc.handle(msg)
    Dr, Ir = ox.search(xq, k)
    assert bytes(ans) == bytes(wire.encode_answer(Ir, Dr, k, b))
    I, D = wire.decode_answer(bytes(ans), k, b)
    np.testing.assert_array_equal(I, Ir)
    np.testing.assert_array_equal(D, Dr)
    # the dict API of FaissServer.retrieve gives the same
    out = svc.retrieve(xq)
    np.testing.assert_array_equal(out["id"], Ir)
    np.testing.assert_array_equal(out["dist"], Dr)


def test_serve_request_with_lists_matches_oracle_preassigned(golden_dir):
    ix, ox, z = golden_pair(golden_dir)
    b, k = 17, 10
    xq = np.ascontiguousarray(z["xq"][:b], np.float32)
    lists = np.ascontiguousarray(z["or_lists"][:b], np.int64)
    lists[3, 1] = -1  # a skipped probe
    lists[5, :] = lists[5, 0]  # a repeated list
    dim, np_ = xq.shape[1], lists.shape[1]
    svc = RetrievalService(ix, batch_size=b, default_k=k, nprobe=np_, request_with_lists=1)
    msg = wire.encode_request_with_lists(xq, lists, b, dim, np_, k)
    assert len(msg) == svc.query_msg_len
    ans = svc.handle(msg)
    I, D = wire.decode_answer(bytes(ans), k, b)
    Dp, Ip = ix.search_preassigned(xq, k, lists)
    np.testing.assert_array_equal(I, Ip)
    np.testing.assert_array_equal(D, Dp)
    ok = [i for i in range(b) if i != 5]  # the oracle scans a repeated list twice (as Faiss)
    Dr, Ir = ox.search_preassigned(xq[ok], k, lists[ok])
    np.testing.assert_array_equal(I[ok], Ir)
    np.testing.assert_array_equal(D[ok], Dr)


def test_serve_trained_index_small_batch():
    # a GPU-trained index, an odd batch and nprobe (the message offsets of odd shapes: tests/test_wire.py)
    rng = np.random.default_rng(5)
    d, nlist, M, b, k, np_ = 24, 16, 8, 3, 5, 4
    xt = rng.random((2000, d), dtype=np.float32)
    ix = faiss.IndexIVFPQ(None, d, nlist, M, 8, device=0)
    ix.niter_coarse = ix.niter_pq = 4
    ix.train(xt)
    ix.add(xt)
    ix.nprobe = np_
    xq = rng.random((b, d), dtype=np.float32)
    _, lists = ix.quantizer.search(xq, np_)
    msg = bytes(wire.encode_request_with_lists(xq, lists, b, d, np_, k))
    ans = ix.serve_request(msg, b, d, with_lists=True, nprobe=np_)
    I, D = wire.decode_answer(bytes(ans), k, b)
    Dp, Ip = ix.search_preassigned(xq, k, lists)
    np.testing.assert_array_equal(I, Ip)
    np.testing.assert_array_equal(D, Dp)


def test_serve_rejects_malformed_requests(golden_dir):
    ix, _, z = golden_pair(golden_dir)
    xq = np.ascontiguousarray(z["xq"][:4], np.float32)
    b, dim = xq.shape
    msg = wire.encode_request(xq, 10, b, dim)
    with pytest.raises(RuntimeError, match="length"):
        ix.serve_request(bytes(msg[:-4]), b, dim)
    with pytest.raises(RuntimeError, match="dim"):
        ix.serve_request(bytes(msg), b, dim + 1)
    bad_k = bytearray(msg)
    bad_k[:4] = (5000).to_bytes(4, "big")
    with pytest.raises(RuntimeError, match="k in the request"):
        ix.serve_request(bytes(bad_k), b, dim)
    with pytest.raises(RuntimeError, match="answer buffer"):
        ix.serve_request(bytes(msg), b, dim, out=bytearray(10))
    lists = np.zeros((b, ix.nprobe), np.int64)
    ml = wire.encode_request_with_lists(xq, lists, b, dim, ix.nprobe, 10)
    bad_hdr = bytes(ml[:4]) + (dim + 1).to_bytes(4, "big") + bytes(ml[8:])  # header dim != server dim
    with pytest.raises(RuntimeError, match="header"):
        ix.serve_request(bad_hdr, b, dim, with_lists=True, nprobe=ix.nprobe)
    lists[1, 2] = ix.nlist + 3
    ml = wire.encode_request_with_lists(xq, lists, b, dim, ix.nprobe, 10)
    with pytest.raises(RuntimeError, match="out of range"):
        ix.serve_request(bytes(ml), b, dim, with_lists=True, nprobe=ix.nprobe)
    svc = RetrievalService(ix, batch_size=b, default_k=5, nprobe=ix.nprobe)
    with pytest.raises(RuntimeError, match="k=10"):
        svc.handle(msg)
    # the index still serves correctly after the errors
    ans = ix.serve_request(bytes(msg), b, dim)
    D, I = ix.search(xq, 10)
    assert bytes(ans) == bytes(wire.encode_answer(I, D, 10, b))


def test_serve_plain_request_honors_nprobe_argument(golden_dir):
    """serve_request(nprobe=p) on a plain request searches with p probes for that
    call only; the index's own nprobe is restored afterwards."""
    ix, ox, z = golden_pair(golden_dir)
    xq = np.ascontiguousarray(z["xq"][:8], np.float32)
    b, dim = xq.shape
    p = int(z["nprobe"])
    ix.nprobe = 1
    ox.nprobe = p
    msg = wire.encode_request(xq, 10, b, dim)
    ans = ix.serve_request(msg, b, dim, nprobe=p)
    Dr, Ir = ox.search(xq, 10)
    assert bytes(ans) == bytes(wire.encode_answer(Ir, Dr, 10, b))
    assert ix.nprobe == 1
