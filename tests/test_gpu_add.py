"""Device-side add (ivfpq_add_device; ivfpq_add routes host buffers through the
same path): coarse assignment on the matrix cores, PQ encode and the merge into
the device list image.  Reference: the 1e9 base set added through the GPU
index in slices, Chameleon/Faiss_experiments/bench_gpu_1bn.py:598-658.

Checked against the oracle's encode (list and code of every vector), the
per-list label order of the image, list-range shards keeping only their own
lists, mixed host/device/pre-encoded adds, and search parity afterwards.
"""
import numpy as np
import pytest

import faiss_amd as faiss
from faiss_amd import datasets
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def trained_pair(d=64, nlist=256, M=16, metric=faiss.METRIC_L2, seed=3):
    xt = datasets.synthetic_sift_like(20_000, d, seed=seed, n_centres=500)
    ix = faiss.index_factory(d, f"IVF{nlist},PQ{M}", metric)
    ix.niter_coarse = ix.niter_pq = 4
    ix.train(xt)
    ox = O.OracleIVFPQ(d, nlist, M, metric=O.METRIC_INNER_PRODUCT if metric == faiss.METRIC_INNER_PRODUCT
                       else O.METRIC_L2)
    ox.set_trained(ix.centroids(), ix.codebook())
    return ix, ox


def lists_of(ix):
    return [(ix.invlists.get_codes(l).reshape(-1, ix.M), ix.invlists.get_ids(l)) for l in range(ix.nlist)]


@pytest.mark.parametrize("metric", [faiss.METRIC_L2, faiss.METRIC_INNER_PRODUCT])
def test_add_device_matches_oracle_encode(metric):
    import torch

    ix, ox = trained_pair(metric=metric)
    xb = datasets.synthetic_sift_like(30_000, 64, seed=11, n_centres=500)
    if metric == faiss.METRIC_INNER_PRODUCT:
        xb = xb - xb.mean(0, keepdims=True)
    # two device adds (sequential ids), the second with a few vectors only
    ix.add_device(torch.from_numpy(xb[:29_000]).cuda())
    ix.add_device(torch.from_numpy(xb[29_000:]).cuda())
    assert ix.ntotal == 30_000
    lo, co = ox.encode(xb)
    for l, (codes, ids) in enumerate(lists_of(ix)):
        assert np.all(np.diff(ids) > 0)  # label-sorted
        np.testing.assert_array_equal(lo[ids], l)
        np.testing.assert_array_equal(codes, co[ids])
    ox.add_preencoded(lo, co, np.arange(30_000, dtype=np.int64))
    ix.nprobe = ox.nprobe = 16
    xq = datasets.synthetic_sift_like(256, 64, seed=12, n_centres=500)
    for k in (10, 100):
        D, I = ix.search(xq, k)
        Dr, Ir = ox.search(xq, k)
        np.testing.assert_array_equal(I, Ir)
        np.testing.assert_array_equal(D, Dr)


def test_add_host_and_device_paths_agree_with_user_ids():
    """Host add_with_ids (shuffled ids), device add with ids, pre-encoded adds,
    in any mix: the lists equal the oracle's (list, code) per label and searches
    equal the oracle."""
    import torch

    ix, ox = trained_pair(seed=5)
    rng = np.random.default_rng(0)
    xb = datasets.synthetic_sift_like(12_000, 64, seed=13, n_centres=500)
    ids = rng.permutation(1_000_000)[:12_000].astype(np.int64)
    ix.add_with_ids(xb[:5000], ids[:5000])
    ix.add_device(torch.from_numpy(xb[5000:9000]).cuda(), torch.from_numpy(ids[5000:9000]).cuda())
    lo, co = ox.encode(xb)
    ix.add_preencoded(lo[9000:], co[9000:], ids[9000:])
    assert ix.ntotal == 12_000
    by_id = {int(i): j for j, i in enumerate(ids)}
    # (host-side appends keep insertion order in the host lists; the device image sorts)
    for l, (codes, lids) in enumerate(lists_of(ix)):
        j = np.array([by_id[int(i)] for i in lids], np.int64)
        np.testing.assert_array_equal(lo[j], l)
        np.testing.assert_array_equal(codes, co[j])
    ox.add_preencoded(lo, co, ids)
    ix.nprobe = ox.nprobe = 8
    xq = datasets.synthetic_sift_like(128, 64, seed=14, n_centres=500)
    D, I = ix.search(xq, 20)
    Dr, Ir = ox.search(xq, 20)
    np.testing.assert_array_equal(I, Ir)
    np.testing.assert_array_equal(D, Dr)


def test_add_device_list_range_shard_keeps_its_lists():
    import torch

    ix, ox = trained_pair(seed=7)
    xb = datasets.synthetic_sift_like(20_000, 64, seed=15, n_centres=500)
    lo, co = ox.encode(xb)
    sh = faiss.IndexIVFPQ(None, 64, 256, 16, 8, device=0)
    sh.set_trained(ix.centroids(), ix.codebook())
    sh.set_list_range(64, 160)
    sh.add_device(torch.from_numpy(xb).cuda())
    keep = (lo >= 64) & (lo < 160)
    assert sh.ntotal == int(keep.sum())
    sizes = sh.invlists.list_sizes()
    assert sizes[:64].sum() == 0 and sizes[160:].sum() == 0
    for l in range(64, 160):
        np.testing.assert_array_equal(sh.invlists.get_ids(l), np.flatnonzero(lo == l))
        np.testing.assert_array_equal(sh.invlists.get_codes(l).reshape(-1, 16), co[lo == l])
    # the range cannot change under pending adds, even when none of them is kept
    # (ntotal == 0 alone let such a change through)
    sh2 = faiss.IndexIVFPQ(None, 64, 256, 16, 8, device=0)
    sh2.set_trained(ix.centroids(), ix.codebook())
    sh2.set_list_range(0, 1)
    far = xb[lo >= 1][:100]
    sh2.add_device(torch.from_numpy(far).cuda())
    assert sh2.ntotal == 0
    with pytest.raises(RuntimeError, match="list range"):
        sh2.set_list_range(0, 256)
    # a reset empties the device image too
    sh.reset()
    assert sh.ntotal == 0 and sh.invlists.list_sizes().sum() == 0
    sh.nprobe = 8
    D, I = sh.search(xb[:4], 5)
    assert (I == -1).all()


def test_add_device_large_nlist_segmented_assignment():
    """nlist >= 8192: the assignment runs the segmented coarse quantizer (no
    [rows x nlist] distance matrix); lists equal the oracle's encode."""
    import torch

    rng = np.random.default_rng(9)
    d, nlist, M = 96, 10_000, 48
    cent = rng.integers(0, 64, size=(nlist, d)).astype(np.float32)
    cb = rng.standard_normal((M, 256, d // M), dtype=np.float32)
    ix = faiss.IndexIVFPQ(None, d, nlist, M, 8, device=0)
    ix.set_trained(cent, cb)
    ox = O.OracleIVFPQ(d, nlist, M)
    ox.set_trained(cent, cb)
    xb = rng.integers(0, 64, size=(40_000, d)).astype(np.float32)
    ix.add_device(torch.from_numpy(xb).cuda())
    lo, co = ox.encode(xb)
    got_l = np.empty(40_000, np.int64)
    got_c = np.empty((40_000, M), np.uint8)
    for l in range(nlist):
        i = ix.invlists.get_ids(l)
        got_l[i] = l
        got_c[i] = ix.invlists.get_codes(l).reshape(-1, M)
    np.testing.assert_array_equal(got_l, lo)
    np.testing.assert_array_equal(got_c, co)


def test_incremental_add_above_65536_lists():
    """The per-list merge of incremental adds (k_merge_lists) at nlist 70 000: its
    grid takes at most 65 535 lists per row of workgroups and strides over the rest
    (ADVICE r04); two device adds with interleaved labels, then every list equals the
    oracle's entries for both chunks, label-sorted."""
    import torch

    rng = np.random.default_rng(21)
    d, nlist, M = 16, 70_000, 8
    cent = rng.integers(0, 64, size=(nlist, d)).astype(np.float32)
    cb = rng.standard_normal((M, 256, d // M), dtype=np.float32)
    ix = faiss.IndexIVFPQ(None, d, nlist, M, 8, device=0)
    ix.set_trained(cent, cb)
    ox = O.OracleIVFPQ(d, nlist, M)
    ox.set_trained(cent, cb)
    n = 200_000
    xb = rng.integers(0, 64, size=(n, d)).astype(np.float32)
    ids = rng.permutation(10 * n)[:n].astype(np.int64)
    half = n // 2
    ix.add_with_ids(xb[:half], ids[:half])
    ix.nprobe = 4
    ix.search(xb[:8], 5)  # the first chunk is merged into the image here
    ix.add_with_ids(xb[half:], ids[half:])
    ix.search(xb[:8], 5)  # the second chunk merges into the existing lists (labels interleave)
    lo, co = ox.encode(xb)
    for l in np.unique(lo)[:: max(1, len(np.unique(lo)) // 500)]:
        sel = np.flatnonzero(lo == l)
        order = np.argsort(ids[sel], kind="stable")
        np.testing.assert_array_equal(ix.invlists.get_ids(int(l)), ids[sel][order])
        np.testing.assert_array_equal(ix.invlists.get_codes(int(l)).reshape(-1, M), co[sel][order])
    assert int(ix.invlists.list_sizes().sum()) == n


@pytest.mark.parametrize("shard", [False, True])
def test_incremental_adds_in_50k_chunks(shard):
    """beir's FaissIndex.build adds in 50k chunks (beir/beir/retrieval/search/
    dense/faiss_index.py:40-42): 8 device and host adds of 50k vectors with
    random user ids (labels interleave across chunks, so the per-list merge
    places new entries between old ones), a search after the third chunk (the
    pending entries are merged into the image then) and list reads at the end.
    Every list holds exactly the oracle's (list, code) per label, label-sorted,
    the shard keeps only its lists, and searches equal the oracle."""
    import torch

    ix, ox = trained_pair(seed=7)
    lo_l, hi_l = (64, 192) if shard else (0, 256)
    ix.set_list_range(lo_l, hi_l)
    rng = np.random.default_rng(3)
    n, ch = 400_000, 50_000
    xb = datasets.synthetic_sift_like(n, 64, seed=17, n_centres=500)
    ids = rng.permutation(10_000_000)[:n].astype(np.int64)
    xq = datasets.synthetic_sift_like(128, 64, seed=18, n_centres=500)
    lo, co = ox.encode(xb)
    keep = (lo >= lo_l) & (lo < hi_l)
    ix.nprobe = ox.nprobe = 24
    for c in range(0, n, ch):
        if (c // ch) % 2 == 0:
            ix.add_device(torch.from_numpy(xb[c:c + ch]).cuda(), torch.from_numpy(ids[c:c + ch]).cuda())
        else:
            ix.add_with_ids(xb[c:c + ch], ids[c:c + ch])
        assert ix.ntotal == int(keep[:c + ch].sum())
        if c == 2 * ch:  # a search between adds merges the pending chunks into the image
            ox2 = O.OracleIVFPQ(64, 256, 16)
            ox2.set_trained(ix.centroids(), ix.codebook())
            k3 = keep[:3 * ch]
            ox2.add_preencoded(lo[:3 * ch][k3], co[:3 * ch][k3], ids[:3 * ch][k3])
            ox2.nprobe = 24
            D, I = ix.search(xq, 10)
            Dr, Ir = ox2.search(xq, 10)
            np.testing.assert_array_equal(I, Ir)
            np.testing.assert_array_equal(D, Dr)
    by_id = {int(i): j for j, i in enumerate(ids)}
    sizes = ix.invlists.list_sizes()
    assert sizes[:lo_l].sum() == 0 and sizes[hi_l:].sum() == 0
    for l, (codes, lids) in enumerate(lists_of(ix)):
        assert np.all(np.diff(lids) > 0)  # label-sorted
        j = np.array([by_id[int(i)] for i in lids], np.int64)
        np.testing.assert_array_equal(lo[j], l)
        np.testing.assert_array_equal(codes, co[j])
    ox.add_preencoded(lo[keep], co[keep], ids[keep])
    for k in (10, 100):
        D, I = ix.search(xq, k)
        Dr, Ir = ox.search(xq, k)
        np.testing.assert_array_equal(I, Ir)
        np.testing.assert_array_equal(D, Dr)
    assert ix.error_count() == 0
