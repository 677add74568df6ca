"""Stale partial lists (DESIGN.md §4 "Tagged partial lists").

Every per-wave partial list is a set of 16-B records tagged with the batch epoch
and the slot; the merges never use an entry whose tag is not this batch's and
rescan its probe instead.  These tests drive that path on purpose (the
fault-injection hook drops the stores of every n-th partial list, as a lost write
would) and run ordered searches beside an unrelated HBM-copy kernel on a side
stream (the r04 failure condition: ~2e-4 of batches lost a probe's candidates).
Every result must equal the oracle's / the search alone, bit for bit, with the
index-check error word at 0.
"""
import numpy as np
import pytest

import faiss_amd as faiss
from faiss_amd import datasets
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _oracle_of(ix, d, nlist, M, nprobe, metric="l2"):
    ox = O.OracleIVFPQ(d, nlist, M, metric=metric) if metric != "l2" else O.OracleIVFPQ(d, nlist, M)
    ox.set_trained(ix.centroids(), ix.codebook())
    for l in range(nlist):
        ox.list_ids[l] = ix.invlists.get_ids(l)
        ox.list_codes[l] = ix.invlists.get_codes(l).reshape(-1, M)
    ox.ntotal = ix.ntotal
    ox.nprobe = nprobe
    return ox


@pytest.fixture(scope="module")
def small_index():
    xt = datasets.synthetic_sift_like(20_000, 64, seed=4321, n_centres=20_000)
    xb = datasets.synthetic_sift_like(100_000, 64, seed=1234, n_centres=20_000)
    xq = datasets.synthetic_sift_like(512, 64, seed=123, n_centres=20_000)
    ix = faiss.index_factory(64, "IVF256,PQ8", device=0)
    ix.niter_coarse = ix.niter_pq = 8
    ix.train(xt)
    ix.add(xb)
    ix.nprobe = 12
    return ix, xq, _oracle_of(ix, 64, 256, 8, 12)


# k = 10: row-packed scan + fast merge; 32: one-row top-k; 100: k_merge_radix;
# 300: k_merge_big; 1000: the 16-row full merge
@pytest.mark.parametrize("k", [10, 32, 100, 300, 1000])
@pytest.mark.parametrize("every", [3, 7])
def test_lost_partial_lists_are_rescanned(small_index, k, every):
    ix, xq, ox = small_index
    Dr, Ir = ox.search(xq, k, 8)
    st0, rp0 = ix.repair_stats()
    ix.set_fault_injection(every)
    try:
        D, I = ix.search(xq, k)
    finally:
        ix.set_fault_injection(0)
    np.testing.assert_array_equal(I, Ir)
    np.testing.assert_array_equal(D, Dr)
    st, rp = ix.repair_stats()
    assert rp > rp0 and st > st0  # the path under test actually ran
    assert ix.error_count() == 0
    D2, I2 = ix.search(xq, k)  # and the next search, without the hook, needs no repair
    np.testing.assert_array_equal(I2, Ir)
    assert ix.repair_stats()[1] == rp


def test_lost_partial_lists_inner_product_and_preassigned():
    xt = datasets.synthetic_sift_like(20_000, 64, seed=7, n_centres=5_000)
    xb = datasets.synthetic_sift_like(60_000, 64, seed=8, n_centres=5_000)
    xq = datasets.synthetic_sift_like(256, 64, seed=9, n_centres=5_000)
    ix = faiss.index_factory(64, "IVF128,PQ16", faiss.METRIC_INNER_PRODUCT, device=0)
    ix.niter_coarse = ix.niter_pq = 6
    ix.train(xt)
    ix.add(xb)
    ix.nprobe = 8
    D0, I0 = ix.search(xq, 20)
    Dq, Iq = ix.quantizer.search(xq, 8)
    P0 = ix.search_preassigned(xq, 20, Iq, Dq)
    ix.set_fault_injection(5)
    try:
        D, I = ix.search(xq, 20)
        P = ix.search_preassigned(xq, 20, Iq, Dq)
    finally:
        ix.set_fault_injection(0)
    np.testing.assert_array_equal(I, I0)
    np.testing.assert_array_equal(D, D0)
    np.testing.assert_array_equal(P[1], P0[1])
    np.testing.assert_array_equal(P[0], P0[0])
    assert ix.repair_stats()[1] > 0
    assert ix.error_count() == 0


def test_lost_partial_lists_nprobe_above_64(small_index):
    ix, xq, _ = small_index
    ix.nprobe = 96
    try:
        D0, I0 = ix.search(xq[:128], 10)
        ix.set_fault_injection(11)
        try:
            D, I = ix.search(xq[:128], 10)
        finally:
            ix.set_fault_injection(0)
    finally:
        ix.nprobe = 12
    np.testing.assert_array_equal(I, I0)
    np.testing.assert_array_equal(D, D0)


@pytest.mark.parametrize("k", [10, 100])
def test_ordered_searches_beside_a_concurrent_copy_kernel(small_index, k):
    """The r04 failure condition, as a gate: one stream of ordered searches while a
    512 MB device-to-device copy loop runs on a side stream.  Every batch must equal
    its search alone (checked against the oracle for the first), and no partial list
    may have been stale: the merge would repair one silently, so a repair here is
    the regression this gate exists to catch (the log of any event is printed)."""
    import torch

    ix, xq, ox = small_index
    nb, rounds = 2, 150
    xd = torch.from_numpy(xq).cuda().view(nb, 256, 64)
    ref = []
    for b in range(nb):
        D, I = ix.search_device(xd[b], k)
        torch.cuda.synchronize()
        ref.append((D.cpu().numpy(), I.cpu().numpy()))
    Do, Io = ox.search(xq[:256], k, 8)
    np.testing.assert_array_equal(ref[0][1], Io)
    np.testing.assert_array_equal(ref[0][0], Do)
    hog_a = torch.empty(1 << 27, device="cuda")
    hog_b = torch.empty_like(hog_a)
    side = torch.cuda.Stream()
    main = torch.cuda.Stream()
    st0 = ix.repair_stats()
    outs = [(torch.empty((256, k), device="cuda"), torch.empty((256, k), dtype=torch.int64, device="cuda"))
            for _ in range(nb * rounds)]
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        for _ in range(rounds // 3):
            hog_b.copy_(hog_a)
    for r in range(rounds):
        for b in range(nb):
            ix.search_device(xd[b], k, *outs[r * nb + b], stream=main.cuda_stream)
    torch.cuda.synchronize()
    bad = [i for i, (D, I) in enumerate(outs)
           if not (np.array_equal(I.cpu().numpy(), ref[i % nb][1]) and np.array_equal(D.cpu().numpy(), ref[i % nb][0]))]
    st = ix.repair_stats()
    print(f"k={k}: stale reads {st[0] - st0[0]}, repairs {st[1] - st0[1]}, log {ix.repair_log(8)}")
    assert not bad, f"{len(bad)} of {len(outs)} batches differ from their search alone"
    assert ix.error_count() == 0
    assert tuple(st) == tuple(st0), f"stale reads / repairs beside the copy loop: {st[0] - st0[0]} / {st[1] - st0[1]}"
