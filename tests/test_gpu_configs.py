"""GPU parity at the BASELINE.json config shapes (C1-C4) and for the list-range
shard path, through the C-ABI, bit-exact against the CPU oracle.

* C1 / C2: bench.py's SIFT1M-shaped index (nb = 1e6, IVF1024,PQ16, 200k-centre
  data, 25 + 25 training iterations) at nprobe 8 and 16.
* C3-shaped: d = 768, M = 64 (64-B codes), nprobe = 32, k in {10, 1000}, at a
  reduced base size (the kernels' M = 64 instantiations).
* C4-shaped: d = 96, M = 48 (dsub 2), nlist = 65536 (the large-nlist coarse
  path), nprobe = 32, at a reduced base size.
* Shards: N in {2, 4} list-range handles on one GPU (set_list_range, as each
  rank of bench.py's shard mode holds), partials merged on the device with
  merge_topk_device; must equal the unsharded result (reference counterpart:
  IndexShards, Chameleon/Faiss_experiments/bench_gpu_1bn.py:605-616, and the
  host argsort merge of bench_multi_cpu_performance_OSDI.py:203-218).
"""
import numpy as np
import pytest

import faiss_amd as faiss
from faiss_amd import datasets
from faiss_amd.sharding import balanced_list_ranges
from oracle import oracle as O

pytestmark = pytest.mark.gpu
RTOL = 1e-4


def assert_same(D, I, Dr, Ir):
    np.testing.assert_array_equal(I, Ir)
    np.testing.assert_allclose(D, Dr, rtol=RTOL, atol=0)
    np.testing.assert_array_equal(D, Dr)


def oracle_like(ix):
    """Oracle index holding exactly the GPU index's trained quantizers and lists."""
    ox = O.OracleIVFPQ(ix.d, ix.nlist, ix.M)
    ox.set_trained(ix.centroids(), ix.codebook())
    for l in range(ix.nlist):
        ox.list_ids[l] = ix.invlists.get_ids(l)
        ox.list_codes[l] = ix.invlists.get_codes(l).reshape(-1, ix.M)
    ox.ntotal = ix.ntotal
    ox.metric = ix.metric_type
    return ox


def build(d, nlist, M, nb, nt, nq, niter, metric=faiss.METRIC_L2, n_centres=10000):
    xt = datasets.synthetic_sift_like(nt, d, seed=4321, n_centres=n_centres)
    xb = datasets.synthetic_sift_like(nb, d, seed=1234, n_centres=n_centres)
    xq = datasets.synthetic_sift_like(nq, d, seed=123, n_centres=n_centres)
    ix = faiss.index_factory(d, f"IVF{nlist},PQ{M}", metric)
    ix.niter_coarse = ix.niter_pq = niter
    ix.train(xt)
    ix.add(xb)
    return ix, xq


@pytest.fixture(scope="module")
def sift1m():
    # bench.py's C2 index exactly: 200k-centre data, 25 + 25 training iterations
    ix, xq = build(128, 1024, 16, 1_000_000, 100_000, 1024, 25, n_centres=200_000)
    return ix, oracle_like(ix), xq


@pytest.mark.parametrize("nprobe", [8, 16])
def test_c1_c2_sift1m_shape(sift1m, nprobe):
    """C1 (nprobe=8) and C2 (nprobe=16) on the 1e6-vector IVF1024,PQ16 index."""
    ix, ox, xq = sift1m
    ix.nprobe = ox.nprobe = nprobe
    D, I = ix.search(xq, 10)
    Dr, Ir = ox.search(xq, 10)
    assert_same(D, I, Dr, Ir)


def test_c2_encode_parity_and_result_shape(sift1m):
    """GPU add (coarse assignment + PQ encode) equals the oracle's encode on a
    slice of the base set; results are sorted, with no duplicate labels."""
    ix, ox, xq = sift1m
    # the first 20k base vectors (the generator draws in blocks of 65536)
    xb = datasets.synthetic_sift_like(65_536, 128, seed=1234, n_centres=200_000)[:20_000]
    lo, co = ox.encode(xb)
    ids0 = np.concatenate([ix.invlists.get_ids(l) for l in range(ix.nlist)])
    lists_all = np.concatenate([np.full(ix.invlists.list_size(l), l) for l in range(ix.nlist)])
    codes_all = np.concatenate([ox.list_codes[l] for l in range(ix.nlist)])
    sel = ids0 < 20_000
    o = np.argsort(ids0[sel])
    np.testing.assert_array_equal(lists_all[sel][o], lo)
    np.testing.assert_array_equal(codes_all[sel][o], co)
    ix.nprobe = 16
    D, I = ix.search(xq, 10)
    assert np.all(np.diff(D, axis=1) >= 0)
    assert all(len(set(r.tolist())) == 10 for r in I)


def test_c2_k100(sift1m):
    """k = 100, the reference's profiling K (MICRO_GPU_profiling)."""
    ix, ox, xq = sift1m
    ix.nprobe = ox.nprobe = 16
    D, I = ix.search(xq[:512], 100)
    Dr, Ir = ox.search(xq[:512], 100)
    assert_same(D, I, Dr, Ir)


@pytest.mark.parametrize("nshards", [2, 4])
def test_list_range_shards_c2(sift1m, nshards):
    """N list-range handles on one GPU, each searching the whole batch on the
    device; the stacked partials merged by merge_topk_device equal the
    unsharded oracle result bit for bit."""
    import torch

    ix, ox, xq = sift1m
    ox.nprobe = 16
    sizes = ix.invlists.list_sizes()
    ranges = balanced_list_ranges(sizes, nshards, ix.M)
    xd = torch.from_numpy(xq).cuda()
    Ds, Is = [], []
    for lo, hi in ranges:
        sh = faiss.IndexIVFPQ(None, ix.d, ix.nlist, ix.M, 8, device=0)
        sh.set_trained(ix.centroids(), ix.codebook())
        sh.set_list_range(lo, hi)
        lists = [l for l in range(lo, hi) if sizes[l]]
        sh.add_preencoded(np.concatenate([np.full(sizes[l], l, np.int64) for l in lists]),
                          np.concatenate([ix.invlists.get_codes(l).reshape(-1, ix.M) for l in lists]),
                          np.concatenate([ix.invlists.get_ids(l) for l in lists]))
        sh.nprobe = 16
        D, I = sh.search_device(xd, 10)
        Ds.append(D)
        Is.append(I)
    D, I = faiss.merge_topk_device(torch.stack(Ds), torch.stack(Is))
    torch.cuda.synchronize()
    Dr, Ir = ox.search(xq, 10)
    assert_same(D.cpu().numpy(), I.cpu().numpy(), Dr, Ir)


@pytest.mark.parametrize("nshards", [2, 4])
def test_list_range_shards_golden(golden_dir, nshards):
    """Golden fixture, list ranges that include empty ranges (owning only empty
    lists) and queries none of whose probes land in a range: those shards
    return all-padding partials, and the slots of their unscanned probes are
    never written (the merge must not read them)."""
    import os

    import torch

    z = dict(np.load(os.path.join(golden_dir, "ivfpq_d128_m16.npz")))
    d, M, nlist, nprobe, k = (int(z[n]) for n in ("d", "M", "nlist", "nprobe", "k"))
    sizes = np.diff(z["list_off"])
    list_no = np.repeat(np.arange(nlist, dtype=np.int64), sizes)
    # an uneven cut: shard 0 owns only list 0, emptied below; the rest split the remainder
    cuts = [0, 1] + [1 + (nlist - 1) * r // (nshards - 1) for r in range(1, nshards - 1)] + [nlist]
    ranges = list(zip(cuts[:-1], cuts[1:]))
    keep_all = list_no != 0  # list 0 receives no vectors
    xd = torch.from_numpy(z["xq"]).cuda()
    Ds, Is = [], []
    for lo, hi in ranges:
        sh = faiss.IndexIVFPQ(None, d, nlist, M, 8, device=0)
        sh.set_trained(z["centroids"], z["codebook"])
        sh.set_list_range(lo, hi)
        sel = keep_all & (list_no >= lo) & (list_no < hi)
        if sel.any():
            sh.add_preencoded(list_no[sel], z["codes"][sel], z["ids"][sel])
        sh.nprobe = nprobe
        D, I = sh.search_device(xd, k)
        Ds.append(D)
        Is.append(I)
    torch.cuda.synchronize()
    assert (Is[0].cpu().numpy() == -1).all()  # the empty shard
    D, I = faiss.merge_topk_device(torch.stack(Ds), torch.stack(Is))
    ox = O.OracleIVFPQ(d, nlist, M)
    ox.set_trained(z["centroids"], z["codebook"])
    ox.add_preencoded(list_no[keep_all], z["codes"][keep_all], z["ids"][keep_all])
    ox.nprobe = nprobe
    Dr, Ir = ox.search(z["xq"], k)
    assert_same(D.cpu().numpy(), I.cpu().numpy(), Dr, Ir)


@pytest.fixture(scope="module")
def c3_shape():
    # BEIR-NQ-shaped: 768-d, 64-B codes; nb reduced to 60k (C3 is 2.68M)
    ix, xq = build(768, 256, 64, 60_000, 20_000, 64, 4, n_centres=2000)
    return ix, oracle_like(ix), xq


@pytest.mark.parametrize("k", [10, 1000])
def test_c3_shape_m64_nprobe32(c3_shape, k):
    ix, ox, xq = c3_shape
    ix.nprobe = ox.nprobe = 32
    D, I = ix.search(xq, k)
    Dr, Ir = ox.search(xq, k)
    assert_same(D, I, Dr, Ir)


@pytest.fixture(scope="module")
def c4_shape():
    # Deep1B-shaped: d = 96, M = 48 (dsub 2), nlist = 65536; nb reduced to 400k (C4 is 1e9)
    ix, xq = build(96, 65536, 48, 400_000, 70_000, 96, 2, n_centres=50000)
    return ix, oracle_like(ix), xq


@pytest.mark.parametrize("k", [10, 100])
def test_c4_shape_m48_nlist65536(c4_shape, k):
    ix, ox, xq = c4_shape
    ix.nprobe = ox.nprobe = 32
    D, I = ix.search(xq, k)
    Dr, Ir = ox.search(xq, k)
    assert_same(D, I, Dr, Ir)


def shard_front(shards, xd, B, tables, check=True):
    """Rank r's front half of bench.py's shard step: the coarse quantizer of its own
    slice (with ``tables``: and T3 of the whole batch in the same launch,
    coarse_tables_device), the probes concatenated (the all_gather), and every rank's
    preassigned scan of the whole batch (consuming its tables token)."""
    import torch

    N = len(shards)
    if tables:
        fr = [shards[r].coarse_tables_device(xd[r * B:(r + 1) * B], xd) for r in range(N)]
        for r in ((0, N - 1) if check else ()):  # the coarse half equals the plain coarse step
            Dc, Ic = shards[r].coarse_device(xd[r * B:(r + 1) * B])
            assert torch.equal(Ic, fr[r][1]) and torch.equal(Dc, fr[r][0])
    else:
        fr = [shards[r].coarse_device(xd[r * B:(r + 1) * B]) + (None,) for r in range(N)]
    Dq = torch.cat([f[0] for f in fr])
    Iq = torch.cat([f[1] for f in fr])
    return Dq, Iq, [f[2] for f in fr]


@pytest.mark.parametrize("nshards,tables", [(2, False), (2, True), (4, True)])
def test_sliced_coarse_allgather_shards_c2(sift1m, nshards, tables):
    """bench.py's shard flow emulated on one GPU: rank r runs the coarse
    quantizer on its own 1024/N-query slice only (tables: with T3 of the whole
    batch in the same launch), the (list, dis0) arrays of all slices are
    concatenated (the all_gather), every rank scans its list range for the whole
    batch with search_preassigned_device, and each slice's N partials are merged
    on the device (the all_to_all + merge).  Must equal the unsharded oracle bit
    for bit."""
    import torch

    ix, ox, xq = sift1m
    ox.nprobe = 16
    ix.nprobe = 16
    sizes = ix.invlists.list_sizes()
    ranges = balanced_list_ranges(sizes, nshards, ix.M)
    xd = torch.from_numpy(xq).cuda()
    B = xd.shape[0] // nshards
    shards = []
    for lo, hi in ranges:
        sh = faiss.IndexIVFPQ(None, ix.d, ix.nlist, ix.M, 8, device=0)
        sh.set_trained(ix.centroids(), ix.codebook())
        sh.set_list_range(lo, hi)
        lists = [l for l in range(lo, hi) if sizes[l]]
        sh.add_preencoded(np.concatenate([np.full(sizes[l], l, np.int64) for l in lists]),
                          np.concatenate([ix.invlists.get_codes(l).reshape(-1, ix.M) for l in lists]),
                          np.concatenate([ix.invlists.get_ids(l) for l in lists]))
        sh.nprobe = 16
        shards.append(sh)
    Dq, Iq, toks = shard_front(shards, xd, B, tables)
    parts = [sh.search_preassigned_device(xd, 10, Iq, Dq, tables=t) for sh, t in zip(shards, toks)]
    Dm, Im = [], []
    for r in range(nshards):  # slice r's partials from every rank, merged
        Ds = torch.stack([p[0][r * B:(r + 1) * B] for p in parts])
        Is = torch.stack([p[1][r * B:(r + 1) * B] for p in parts])
        D, I = faiss.merge_topk_device(Ds, Is)
        Dm.append(D)
        Im.append(I)
    torch.cuda.synchronize()
    Dr, Ir = ox.search(xq, 10)
    assert_same(torch.cat(Dm).cpu().numpy(), torch.cat(Im).cpu().numpy(), Dr, Ir)


@pytest.mark.parametrize("nq,nprobe,metric,gauss", [(1, 1, 1, 0), (17, 33, 1, 0), (1000, 64, 1, 0), (200, 32, 1, 1),
                                                     (130, 16, 0, 1)])
def test_segmented_coarse_matches_oracle(nq, nprobe, metric, gauss):
    """nlist >= 8192 takes the segmented coarse quantizer (per-segment top-nprobe
    on the matrix cores, no [nq][nlist] key matrix); nlist = 20000 leaves a
    partial last tile, and the batch sizes give 1 to many segments per query.
    From 64 queries on the segments are walked by 64-query tiles
    (k_coarse_segtop_tiled); Gaussian data tests its rounding order, and the
    inner-product case its IP keys."""
    import torch

    rng = np.random.default_rng(7)
    d, nlist, M = 96, 20000, 48
    if gauss:
        cent = rng.standard_normal((nlist, d), dtype=np.float32)
    else:
        cent = rng.integers(0, 64, size=(nlist, d)).astype(np.float32)
    cent[123] = cent[456]  # an exact tie: ordered by list id
    ix = faiss.IndexIVFPQ(None, d, nlist, M, 8, metric, device=0)
    ix.set_trained(cent, rng.standard_normal((M, 256, d // M), dtype=np.float32))
    ix.nprobe = nprobe
    if gauss:
        xq = rng.standard_normal((nq, d), dtype=np.float32)
    else:
        xq = rng.integers(0, 64, size=(nq, d)).astype(np.float32)
    Dq, Iq = ix.coarse_device(torch.from_numpy(xq).cuda())
    Dr, Ir = O.coarse_search(xq, cent, nprobe, metric=metric)
    np.testing.assert_array_equal(Iq.cpu().numpy(), Ir)
    np.testing.assert_array_equal(Dq.cpu().numpy(), Dr)


@pytest.mark.parametrize("d,nlist,nq,metric", [(768, 4096, 200, 1), (264, 1102, 64, 1), (768, 1500, 129, 0),
                                               (256, 2048, 1000, 0)])
def test_tiled_coarse_matches_oracle(d, nlist, nq, metric):
    """d >= 256 with 1024 < nlist < 8192 takes the 64-query x 128-centroid tiled
    key GEMM (C3's coarse step); d = 264 leaves a partial k-chunk, nlist = 1102 a
    partial centroid tile and a padded transposed row, nq = 129 / 200 a partial
    query tile.  Gaussian data, so the keys' rounding order is what is tested."""
    import torch

    rng = np.random.default_rng(11)
    M = 8
    cent = rng.standard_normal((nlist, d), dtype=np.float32)
    cent[77] = cent[901]  # an exact tie: ordered by list id
    ix = faiss.IndexIVFPQ(None, d, nlist, M, 8, metric, device=0)
    ix.set_trained(cent, rng.standard_normal((M, 256, d // M), dtype=np.float32))
    ix.nprobe = 32
    xq = rng.standard_normal((nq, d), dtype=np.float32)
    Dq, Iq = ix.coarse_device(torch.from_numpy(xq).cuda())
    Dr, Ir = O.coarse_search(xq, cent, 32, metric=metric)
    np.testing.assert_array_equal(Iq.cpu().numpy(), Ir)
    np.testing.assert_array_equal(Dq.cpu().numpy(), Dr)


@pytest.mark.parametrize("k", [10, 100])
def test_c4_shape_eight_list_range_shards(c4_shape, k):
    """C4's list-sharded form at its shape (d 96, M 48, nlist 65536, nprobe 32)
    on one GPU: 8 list-range handles, each running the segmented coarse
    quantizer on its own query slice, the probes concatenated (the all_gather),
    each scanning its lists for the whole batch, and each slice's 8 partials
    merged on the device (the all_to_all + merge).  Must equal the unsharded
    oracle bit for bit (reference: IndexShards over 8 GPUs,
    bench_gpu_1bn.py:605-616)."""
    import torch

    ix, ox, xq = c4_shape
    N = 8
    ox.nprobe = 32
    sizes = ix.invlists.list_sizes()
    ranges = balanced_list_ranges(sizes, N, ix.M)
    xd = torch.from_numpy(xq).cuda()
    B = xd.shape[0] // N
    shards = []
    for lo, hi in ranges:
        sh = faiss.IndexIVFPQ(None, ix.d, ix.nlist, ix.M, 8, device=0)
        sh.set_trained(ix.centroids(), ix.codebook())
        sh.set_list_range(lo, hi)
        lists = [l for l in range(lo, hi) if sizes[l]]
        if lists:
            sh.add_preencoded(np.concatenate([np.full(sizes[l], l, np.int64) for l in lists]),
                              np.concatenate([ix.invlists.get_codes(l).reshape(-1, ix.M) for l in lists]),
                              np.concatenate([ix.invlists.get_ids(l) for l in lists]))
        sh.nprobe = 32
        shards.append(sh)
    Dq, Iq, toks = shard_front(shards, xd, B, tables=k == 10)  # (the segmented coarse launch + its T3 launch)
    parts = [sh.search_preassigned_device(xd, k, Iq, Dq, tables=t) for sh, t in zip(shards, toks)]
    Dm, Im = [], []
    for r in range(N):
        D, I = faiss.merge_topk_device(torch.stack([p[0][r * B:(r + 1) * B] for p in parts]),
                                       torch.stack([p[1][r * B:(r + 1) * B] for p in parts]))
        Dm.append(D)
        Im.append(I)
    torch.cuda.synchronize()
    del shards, parts
    Dr, Ir = ox.search(xq, k)
    assert_same(torch.cat(Dm).cpu().numpy(), torch.cat(Im).cpu().numpy(), Dr, Ir)


def test_precomputed_tables_on_a_side_stream(sift1m):
    """bench.py's shard step computes T3 of the global batch on a side stream
    (precompute_tables_device) while the coarse step runs; the preassigned search
    given that call's token then uses it.  Results equal the plain preassigned
    search and the oracle, over several back-to-back steps (the next step's T3
    is ordered after the previous search that read the buffer).  Tables are
    handed over only by token: a search without one never uses pending tables,
    a consumed, overwritten or mis-sized token is rejected, and retraining drops
    pending tables."""
    import torch

    ix, ox, xq = sift1m
    ix.nprobe = ox.nprobe = 16
    xd = torch.from_numpy(xq).cuda()
    Dq, Iq = ix.coarse_device(xd)
    Dr, Ir = ox.search(xq, 10)
    side = torch.cuda.Stream()
    for step in range(3):
        side.wait_stream(torch.cuda.current_stream())
        tok = ix.precompute_tables_device(xd, stream=side.cuda_stream)
        D, I = ix.search_preassigned_device(xd, 10, Iq, Dq, tables=tok)
        torch.cuda.synchronize()
        assert_same(D.cpu().numpy(), I.cpu().numpy(), Dr, Ir)
        with pytest.raises(RuntimeError, match="not pending"):  # consumed
            ix.search_preassigned_device(xd, 10, Iq, Dq, tables=tok)
    # tables of other queries, pending under the same pointer, are not used by a search without the token
    x2 = torch.from_numpy(xq[::-1].copy()).cuda()
    xd_alias = xd.clone()
    xd.copy_(x2)
    tok = ix.precompute_tables_device(xd, stream=side.cuda_stream)
    xd.copy_(xd_alias)
    torch.cuda.synchronize()
    D, I = ix.search_preassigned_device(xd, 10, Iq, Dq)
    torch.cuda.synchronize()
    assert_same(D.cpu().numpy(), I.cpu().numpy(), Dr, Ir)
    with pytest.raises(RuntimeError, match="computed for"):  # token of n queries used for another n
        ix.search_preassigned_device(xd[:512].contiguous(), 10, Iq[:512].contiguous(), Dq[:512].contiguous(),
                                     tables=tok)
    # a fourth pending precompute overwrites the oldest token
    toks = [ix.precompute_tables_device(xd, stream=side.cuda_stream) for _ in range(3)]
    with pytest.raises(RuntimeError, match="not pending"):
        ix.search_preassigned_device(xd, 10, Iq, Dq, tables=tok)
    D, I = ix.search_preassigned_device(xd, 10, Iq, Dq, tables=toks[0])
    torch.cuda.synchronize()
    assert_same(D.cpu().numpy(), I.cpu().numpy(), Dr, Ir)
    ix.set_trained(ix.centroids(), ix.codebook())  # new quantizers: pending tables are dropped
    with pytest.raises(RuntimeError, match="not pending"):
        ix.search_preassigned_device(xd, 10, Iq, Dq, tables=toks[1])
    assert ix.error_count() == 0


@pytest.mark.parametrize("inflight", [False, True])
def test_precomputed_tables_with_batches_in_flight(sift1m, inflight):
    """The shard step pipelined: 8 batches (4 distinct query sets) issued on 2
    compute streams, each with its own side stream for the T3 ahead, and with the
    T3 of batch s + 1 issued before the search of batch s, with no
    synchronisation, in both stream modes (ordered, and batches in flight).
    Every batch equals its plain preassigned search."""
    import torch

    ix, ox, xq = sift1m
    ix.nprobe = 16
    B = 256
    xs = [torch.from_numpy(xq[i * B:(i + 1) * B]).cuda() for i in range(4)]
    ref = []
    for x in xs:
        Dq, Iq = ix.coarse_device(x)
        D, I = ix.search_preassigned_device(x, 10, Iq, Dq)
        torch.cuda.synchronize()
        ref.append((D.cpu().numpy(), I.cpu().numpy()))
    comp = [torch.cuda.Stream() for _ in range(2)]
    side = [torch.cuda.Stream() for _ in range(2)]
    ix.inflight = inflight
    try:
        torch.cuda.synchronize()
        outs = []
        toks = {0: ix.precompute_tables_device(xs[0], stream=side[0].cuda_stream)}
        for s in range(8):
            j = s % 2
            x = xs[s % 4]
            if s + 1 < 8:  # the next batch's tables first
                toks[s + 1] = ix.precompute_tables_device(xs[(s + 1) % 4], stream=side[(s + 1) % 2].cuda_stream)
            with torch.cuda.stream(comp[j]):
                Dq, Iq = ix.coarse_device(x)
                outs.append(ix.search_preassigned_device(x, 10, Iq, Dq, tables=toks[s]))
        torch.cuda.synchronize()
    finally:
        ix.inflight = False
    for s, (D, I) in enumerate(outs):
        assert_same(D.cpu().numpy(), I.cpu().numpy(), *ref[s % 4])
    assert ix.error_count() == 0


def test_shard_step_pipelined_on_two_streams(sift1m):
    """bench.py's shard loop on one GPU, as its ranks issue it at N = 2: per step
    on stream s % 2, the previous batch of that stream is exchanged and merged
    first, then this batch's front half (coarse of the own slice + T3 of the
    global batch in one launch, probes concatenated, preassigned scans consuming
    the tables token) -- no side stream, no host synchronisation, batches in
    flight.  Every merged batch equals the unsharded oracle."""
    import torch

    ix, ox, xq = sift1m
    ix.nprobe = ox.nprobe = 16
    N, Bg = 2, 512
    sizes = ix.invlists.list_sizes()
    shards = []
    for lo, hi in balanced_list_ranges(sizes, N, ix.M):
        sh = faiss.IndexIVFPQ(None, ix.d, ix.nlist, ix.M, 8, device=0)
        sh.set_trained(ix.centroids(), ix.codebook())
        sh.set_list_range(lo, hi)
        lists = [l for l in range(lo, hi) if sizes[l]]
        sh.add_preencoded(np.concatenate([np.full(sizes[l], l, np.int64) for l in lists]),
                          np.concatenate([ix.invlists.get_codes(l).reshape(-1, ix.M) for l in lists]),
                          np.concatenate([ix.invlists.get_ids(l) for l in lists]))
        sh.nprobe = 16
        sh.inflight = True
        shards.append(sh)
    xs = [torch.from_numpy(xq[i * Bg:(i + 1) * Bg]).cuda() for i in range(2)]
    B = Bg // N
    streams = [torch.cuda.Stream() for _ in range(2)]
    pend, merged = [None, None], []

    def back(j):
        b, parts = pend[j]
        pend[j] = None
        with torch.cuda.stream(streams[j]):
            for r in range(N):
                merged.append((b, r, faiss.merge_topk_device(
                    torch.stack([p[0][r * B:(r + 1) * B] for p in parts]),
                    torch.stack([p[1][r * B:(r + 1) * B] for p in parts]))))

    torch.cuda.synchronize()
    for s in range(8):
        j = s % 2
        if pend[j] is not None:
            back(j)
        x = xs[s % 2]
        with torch.cuda.stream(streams[j]):
            Dq, Iq, toks = shard_front(shards, x, B, tables=True, check=False)
            parts = [sh.search_preassigned_device(x, 10, Iq, Dq, tables=t) for sh, t in zip(shards, toks)]
        pend[j] = (s % 2, parts)
    for j in range(2):
        if pend[j] is not None:
            back(j)
    torch.cuda.synchronize()
    ref = [ox.search(xq[i * Bg:(i + 1) * Bg], 10) for i in range(2)]
    assert len(merged) == 8 * N
    for b, r, (D, I) in merged:
        assert_same(D.cpu().numpy(), I.cpu().numpy(), ref[b][0][r * B:(r + 1) * B], ref[b][1][r * B:(r + 1) * B])
    for sh in shards:
        assert sh.error_count() == 0 and sh.repair_stats() == (0, 0)
