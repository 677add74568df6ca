"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle.

The bar (BASELINE.json north_star): returned IDs bit-exact, L2 distances within
1e-4 relative.  Because the kernels follow the oracle's fp32 operation order,
these tests assert the stronger property where it holds: identical IDs AND
identical distances (np.array_equal), with the 1e-4 tolerance asserted as well.
"""
import os

import numpy as np
import pytest

import faiss_amd as faiss
from faiss_amd import datasets
from oracle import oracle as O

pytestmark = pytest.mark.gpu

CASES = ["d128_m16", "d64_m32_dsub2", "d96_m8_dsub12"]
RTOL = 1e-4  # north_star distance tolerance


def load_case(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, f"ivfpq_{name}.npz")))


def gpu_index(z):
    d, M, nlist = int(z["d"]), int(z["M"]), int(z["nlist"])
    ix = faiss.IndexIVFPQ(None, d, nlist, M, 8, device=0)
    ix.set_trained(z["centroids"], z["codebook"])
    off = z["list_off"]
    list_no = np.repeat(np.arange(nlist, dtype=np.int64), np.diff(off))
    ix.add_preencoded(list_no, z["codes"], z["ids"])
    ix.nprobe = int(z["nprobe"])
    return ix


def oracle_index(z):
    d, M, nlist = int(z["d"]), int(z["M"]), int(z["nlist"])
    ox = O.OracleIVFPQ(d, nlist, M)
    ox.set_trained(z["centroids"], z["codebook"])
    off = z["list_off"]
    list_no = np.repeat(np.arange(nlist, dtype=np.int64), np.diff(off))
    ox.add_preencoded(list_no, z["codes"], z["ids"])
    ox.nprobe = int(z["nprobe"])
    return ox


def assert_same(D, I, Dr, Ir):
    np.testing.assert_array_equal(I, Ir)
    np.testing.assert_allclose(D, Dr, rtol=RTOL, atol=0)
    np.testing.assert_array_equal(D, Dr)


@pytest.mark.parametrize("case", CASES)
def test_search_matches_golden(golden_dir, case):
    z = load_case(golden_dir, case)
    ix = gpu_index(z)
    D, I = ix.search(z["xq"], int(z["k"]))
    assert_same(D, I, z["or_D"], z["or_I"])


@pytest.mark.parametrize("case", CASES)
def test_coarse_and_tables_match_oracle(golden_dir, case):
    import torch

    z = load_case(golden_dir, case)
    ix = gpu_index(z)
    xq = torch.from_numpy(z["xq"]).cuda()
    Dq, Iq = ix.coarse_device(xq)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(Iq.cpu().numpy(), z["or_lists"])
    np.testing.assert_array_equal(Dq.cpu().numpy(), z["or_dis0"])
    T1 = ix.precomputed_table.reshape(int(z["nlist"]), int(z["M"]), 256)
    np.testing.assert_array_equal(T1, O.precompute_T1(z["centroids"], z["codebook"]))


@pytest.mark.parametrize("k", [1, 7, 63, 64, 65, 100, 128, 129, 257, 600, 1024])
def test_k_sweep(golden_dir, k):
    z = load_case(golden_dir, "d128_m16")
    ix, ox = gpu_index(z), oracle_index(z)
    for nprobe in (1, 8):
        ix.nprobe = ox.nprobe = nprobe
        D, I = ix.search(z["xq"], k)
        Dr, Ir = ox.search(z["xq"], k)
        assert_same(D, I, Dr, Ir)


def test_nprobe_above_nlist_is_clamped(golden_dir):
    z = load_case(golden_dir, "d64_m32_dsub2")
    ix, ox = gpu_index(z), oracle_index(z)
    ix.nprobe = 100  # nlist = 32
    ox.nprobe = 32
    D, I = ix.search(z["xq"], 20)
    Dr, Ir = ox.search(z["xq"], 20)
    assert_same(D, I, Dr, Ir)


def test_search_preassigned(golden_dir):
    z = load_case(golden_dir, "d128_m16")
    ix, ox = gpu_index(z), oracle_index(z)
    lists = z["or_lists"].copy()
    dis0 = z["or_dis0"].copy()
    D, I = ix.search_preassigned(z["xq"], 10, lists, dis0)
    assert_same(D, I, z["or_D"], z["or_I"])
    # Dq = None means zeros (upstream contrib default)
    D, I = faiss.contrib.ivf_tools.search_preassigned(ix, z["xq"], 10, lists)
    Dr, Ir = ox.search_preassigned(z["xq"], 10, lists, None)
    assert_same(D, I, Dr, Ir)
    # skipped probes (-1) and the 8-argument Faiss form
    lists[:, ::2] = -1
    D = np.empty((lists.shape[0], 10), np.float32)
    I = np.empty((lists.shape[0], 10), np.int64)
    n = lists.shape[0]
    ix.search_preassigned(n, faiss.swig_ptr(z["xq"]), 10, faiss.swig_ptr(lists), faiss.swig_ptr(dis0),
                          faiss.swig_ptr(D), faiss.swig_ptr(I), False)
    Dr, Ir = ox.search_preassigned(z["xq"], 10, lists, dis0)
    assert_same(D, I, Dr, Ir)


def test_padding_when_fewer_than_k():
    rng = np.random.default_rng(5)
    d, M, nlist = 32, 8, 16
    cent = rng.normal(size=(nlist, d)).astype(np.float32) * 4
    cb = rng.normal(size=(M, 256, d // M)).astype(np.float32)
    ix = faiss.IndexIVFPQ(None, d, nlist, M, 8, device=0)
    ix.set_trained(cent, cb)
    ox = O.OracleIVFPQ(d, nlist, M)
    ox.set_trained(cent, cb)
    x = rng.normal(size=(40, d)).astype(np.float32) * 4
    ix.add(x)
    ox.add(x)
    ix.nprobe = ox.nprobe = 2
    q = rng.normal(size=(9, d)).astype(np.float32) * 4
    D, I = ix.search(q, 30)
    Dr, Ir = ox.search(q, 30)
    assert_same(D, I, Dr, Ir)
    assert (I == -1).any()
    assert np.all(D[I == -1] == np.finfo(np.float32).max)
    # empty index: all padding
    ix.reset()
    D, I = ix.search(q, 5)
    assert np.all(I == -1)
    # zero queries
    D, I = ix.search(np.zeros((0, d), np.float32), 5)
    assert D.shape == (0, 5)


def test_exact_ties_ordered_by_label():
    # duplicate vectors produce identical codes and distances: order is (dist, label)
    rng = np.random.default_rng(11)
    d, M, nlist = 32, 8, 4
    cent = rng.normal(size=(nlist, d)).astype(np.float32)
    cb = rng.normal(size=(M, 256, d // M)).astype(np.float32) * 0.3
    base = rng.normal(size=(20, d)).astype(np.float32)
    x = np.repeat(base, 40, axis=0)
    ids = rng.permutation(x.shape[0]).astype(np.int64) * 3 + 1
    ix = faiss.IndexIVFPQ(None, d, nlist, M, 8, device=0)
    ix.set_trained(cent, cb)
    ox = O.OracleIVFPQ(d, nlist, M)
    ox.set_trained(cent, cb)
    ix.add_with_ids(x, ids)
    ox.add_with_ids(x, ids)
    ix.nprobe = ox.nprobe = 4
    D, I = ix.search(base[:6], 100)
    Dr, Ir = ox.search(base[:6], 100)
    assert_same(D, I, Dr, Ir)


def test_train_and_encode_match_oracle():
    x = datasets.synthetic_sift_like(6000, 32, seed=7, n_centres=50)
    ix = faiss.IndexIVFPQ(None, 32, 16, 8, 8, device=0)
    ix.niter_coarse, ix.niter_pq, ix.seed = 6, 5, 99
    ix.train(x)
    ox = O.OracleIVFPQ(32, 16, 8)
    ox.train(x, niter_coarse=6, niter_pq=5, seed=99)
    np.testing.assert_array_equal(ix.centroids(), ox.centroids)
    np.testing.assert_array_equal(ix.codebook(), ox.codebook)
    xa = datasets.synthetic_sift_like(3000, 32, seed=8, n_centres=50)
    ix.add(xa)
    ox.add(xa)
    for l in range(16):
        np.testing.assert_array_equal(ix.invlists.get_ids(l), ox.list_ids[l])
        np.testing.assert_array_equal(ix.invlists.get_codes(l).reshape(-1, 8), ox.list_codes[l])
    assert ix.ntotal == 3000
    assert ix.quantizer.ntotal == 16


def test_search_after_gpu_training_with_stale_workspaces():
    """The smoke() shape: an index trained on the GPU (whose freed k-means buffers
    leave non-zero memory behind) and searched at once, with probes landing on
    lists that receive no codes.  Partial-result slots of unscanned probes are
    never written, so the merge must not dereference them."""
    xt = datasets.synthetic_sift_like(4000, 64, seed=4321, n_centres=100)
    xb = datasets.synthetic_sift_like(20000, 64, seed=1234, n_centres=100)
    xq = datasets.synthetic_sift_like(64, 64, seed=123, n_centres=100)
    ix = faiss.index_factory(64, "IVF64,PQ16", device=0)
    ix.niter_coarse = ix.niter_pq = 5
    ix.train(xt)
    ix.add(xb)
    ix.nprobe = 8
    D, I = ix.search(xq, 10)
    ox = O.OracleIVFPQ(64, 64, 16)
    ox.set_trained(ix.centroids(), ix.codebook())
    ox.add(xb)
    ox.nprobe = 8
    Dr, Ir = ox.search(xq, 10)
    assert_same(D, I, Dr, Ir)


def test_device_entry_points_match_host(golden_dir):
    import torch

    z = load_case(golden_dir, "d128_m16")
    ix = gpu_index(z)
    xq = torch.from_numpy(z["xq"]).cuda()
    D, I = ix.search_device(xq, 10)
    torch.cuda.synchronize()
    assert_same(D.cpu().numpy(), I.cpu().numpy(), z["or_D"], z["or_I"])
    Dq, Iq = ix.coarse_device(xq)
    D2, I2 = ix.search_preassigned_device(xq, 10, Iq, Dq)
    torch.cuda.synchronize()
    assert_same(D2.cpu().numpy(), I2.cpu().numpy(), z["or_D"], z["or_I"])


def test_device_searches_on_two_streams_without_sync(golden_dir):
    """Two device searches on different streams and then a host search(), with
    no synchronisation in between: the library orders them on the handle's
    shared workspaces (bucket counters, partial lists, T3), so all three are
    bit-exact."""
    import torch

    z = load_case(golden_dir, "d128_m16")
    ix = gpu_index(z)
    xq = torch.from_numpy(z["xq"]).cuda()
    xr = torch.flip(xq, dims=[0]).contiguous()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    outs = []
    for rep in range(3):
        with torch.cuda.stream(s1):
            D1, I1 = ix.search_device(xq, 10)
        with torch.cuda.stream(s2):
            D2, I2 = ix.search_device(xr, 10)
        D3, I3 = ix.search(z["xq"], 10)
        outs.append((D1, I1, D2, I2, D3, I3))
    torch.cuda.synchronize()
    for D1, I1, D2, I2, D3, I3 in outs:
        assert_same(D1.cpu().numpy(), I1.cpu().numpy(), z["or_D"], z["or_I"])
        assert_same(D2.cpu().numpy(), I2.cpu().numpy(), z["or_D"][::-1], z["or_I"][::-1])
        assert_same(D3, I3, z["or_D"], z["or_I"])


@pytest.fixture(scope="module")
def rr_index():
    xt = datasets.synthetic_sift_like(20_000, 64, seed=4321, n_centres=20_000)
    xb = datasets.synthetic_sift_like(100_000, 64, seed=1234, n_centres=20_000)
    xq = datasets.synthetic_sift_like(24 * 256, 64, seed=123, n_centres=20_000)
    ix = faiss.index_factory(64, "IVF256,PQ8", device=0)
    ix.niter_coarse = ix.niter_pq = 8
    ix.train(xt)
    ix.add(xb)
    ix.nprobe = 12
    return ix, xq


@pytest.mark.parametrize("inflight", [False, True])
def test_batches_in_flight_on_round_robin_streams(rr_index, inflight):
    """24 batches issued round robin on 2, 3, 4 and 5 streams with no
    synchronisation, at k = 10 (row-packed scan) and k = 100 (k > 64 merge), with
    a coarse_device + preassigned search interleaved, in both stream modes:
    searches ordered across streams, and batches in flight (k = 10: up to three
    overlapping in per-stream workspaces, 4 and 5 streams take workspaces over).
    Every batch equals its search alone on one stream, bit for bit (those are
    checked against the oracle for the first batch), and the merge kernels'
    index checks count nothing."""
    import torch

    ix, xq = rr_index
    nb = 24
    xd = torch.from_numpy(xq).cuda().view(nb, 256, 64)
    torch.cuda.synchronize()
    for k in (10, 100):
        ref = []
        for b in range(nb):
            D, I = ix.search_device(xd[b], k)
            torch.cuda.synchronize()
            ref.append((D.cpu().numpy(), I.cpu().numpy()))
        if k == 10:
            ox = O.OracleIVFPQ(64, 256, 8)
            ox.set_trained(ix.centroids(), ix.codebook())
            for l in range(256):
                ox.list_ids[l] = ix.invlists.get_ids(l)
                ox.list_codes[l] = ix.invlists.get_codes(l).reshape(-1, 8)
            ox.ntotal = ix.ntotal
            ox.nprobe = 12
            Do, Io = ox.search(xq[:256], k, 4)
            assert_same(ref[0][0], ref[0][1], Do, Io)
        for nst in (2, 3, 4, 5):
            streams = [torch.cuda.Stream() for _ in range(nst)]
            outs = [(torch.empty((256, k), device="cuda"), torch.empty((256, k), dtype=torch.int64, device="cuda"))
                    for _ in range(nb)]
            pre = None
            ix.inflight = inflight
            try:
                torch.cuda.synchronize()
                for b in range(nb):
                    st = streams[b % nst].cuda_stream
                    if b == 5:  # a coarse step + preassigned search in the middle of the pipeline
                        with torch.cuda.stream(streams[b % nst]):
                            Dq, Iq = ix.coarse_device(xd[b], stream=st)
                            pre = ix.search_preassigned_device(xd[b], k, Iq, Dq, stream=st)
                    ix.search_device(xd[b], k, outs[b][0], outs[b][1], stream=st)
                torch.cuda.synchronize()
            finally:
                ix.inflight = False
            for b in range(nb):
                np.testing.assert_array_equal(outs[b][1].cpu().numpy(), ref[b][1], err_msg=f"k={k} streams={nst} b={b}")
                np.testing.assert_array_equal(outs[b][0].cpu().numpy(), ref[b][0], err_msg=f"k={k} streams={nst} b={b}")
            np.testing.assert_array_equal(pre[1].cpu().numpy(), ref[5][1])
            np.testing.assert_array_equal(pre[0].cpu().numpy(), ref[5][0])
    assert ix.error_count() == 0


@pytest.mark.parametrize("k,nst", [(10, 3), (100, 2), (100, 3)])
def test_batches_in_flight_stress(rr_index, k, nst):
    """The concurrent-kernel regression ("Uniform bounds"): 40
    rounds of 24 batches in flight on nst streams -- before the wave-uniform bound fix
    about 1 batch in 1700 (k = 10, 3 streams) to 1 in 60 (k = 100, 2 streams) lost a
    true neighbour here (profiles/r05_ab/, profiles/r05_race_inflight.jsonl).  Every
    batch must equal its search alone, with no index-check or stale-entry events."""
    import torch

    ix, xq = rr_index
    nb = 24
    xd = torch.from_numpy(xq).cuda().view(nb, 256, 64)
    ref = []
    for b in range(nb):
        D, I = ix.search_device(xd[b], k)
        torch.cuda.synchronize()
        ref.append((D.cpu().numpy(), I.cpu().numpy()))
    streams = [torch.cuda.Stream() for _ in range(nst)]
    e0 = ix.error_count()
    rs0 = ix.repair_stats()
    bad = []
    for rnd in range(40):
        outs = [(torch.empty((256, k), device="cuda"), torch.empty((256, k), dtype=torch.int64, device="cuda"))
                for _ in range(nb)]
        ix.inflight = True
        try:
            torch.cuda.synchronize()
            for b in range(nb):
                ix.search_device(xd[b], k, outs[b][0], outs[b][1], stream=streams[b % nst].cuda_stream)
            torch.cuda.synchronize()
        finally:
            ix.inflight = False
        for b in range(nb):
            if not (np.array_equal(outs[b][1].cpu().numpy(), ref[b][1])
                    and np.array_equal(outs[b][0].cpu().numpy(), ref[b][0])):
                bad.append((rnd, b))
    assert not bad, f"{len(bad)} of {40 * nb} batches differ: {bad[:8]}"
    assert ix.error_count() == e0
    # the merge repairs a stale partial list silently (results stay exact), so the
    # gate also requires that no repair happened: a stale read is a regression
    rs = ix.repair_stats()
    assert rs == rs0, f"stale reads / repairs during the stress: {rs[0] - rs0[0]} / {rs[1] - rs0[1]}, " \
                      f"log {ix.repair_log(8)}"


def test_device_entry_points_reject_bad_tensors(golden_dir):
    import torch

    z = load_case(golden_dir, "d128_m16")
    ix = gpu_index(z)
    xq = torch.from_numpy(z["xq"]).cuda()
    for bad in (xq.half(), xq[:, :64], xq.t(), xq.cpu(), xq[:, ::2]):
        with pytest.raises(RuntimeError):
            ix.search_device(bad, 10)
    with pytest.raises(RuntimeError):
        ix.search_device(xq, 10, D=torch.empty((3, 10), device="cuda"))
    Dq, Iq = ix.coarse_device(xq)
    with pytest.raises(RuntimeError):
        ix.search_preassigned_device(xq, 10, Iq.int(), Dq)
    with pytest.raises(RuntimeError):
        ix.search_preassigned_device(xq, 10, Iq[:, :3].contiguous(), None)


def test_merge_topk_device():
    import torch

    rng = np.random.default_rng(3)
    S, n, k = 4, 33, 17
    Ds = np.sort(rng.integers(0, 50, size=(S, n, k)).astype(np.float32), axis=2)
    Is = rng.integers(0, 1000, size=(S, n, k)).astype(np.int64)
    Is[:, :, -2:] = -1
    Ds[:, :, -2:] = np.finfo(np.float32).max
    # make each partial list sorted by (dist, id)
    for s in range(S):
        for q in range(n):
            o = np.lexsort((np.where(Is[s, q] < 0, np.iinfo(np.int64).max, Is[s, q]), Ds[s, q]))
            Ds[s, q], Is[s, q] = Ds[s, q][o], Is[s, q][o]
    D, I = faiss.merge_topk_device(torch.from_numpy(Ds).cuda(), torch.from_numpy(Is).cuda())
    D, I = D.cpu().numpy(), I.cpu().numpy()
    for q in range(n):
        dd = Ds[:, q].reshape(-1)
        ii = Is[:, q].reshape(-1)
        key = np.where(ii < 0, np.iinfo(np.int64).max, ii)
        o = np.lexsort((key, dd))[:k]
        np.testing.assert_array_equal(D[q], dd[o])
        np.testing.assert_array_equal(I[q], ii[o])


def test_flat_search_exact():
    rng = np.random.default_rng(2)
    xb = rng.integers(0, 20, size=(3000, 24)).astype(np.float32)
    xq = rng.integers(0, 20, size=(50, 24)).astype(np.float32)
    fl = faiss.IndexFlatL2(24, device=0)
    fl.add(xb)
    D, I = fl.search(xq, 12)
    dd = ((xq[:, None, :].astype(np.float64) - xb[None, :, :]) ** 2).sum(-1)
    for q in range(xq.shape[0]):
        o = np.lexsort((np.arange(xb.shape[0]), dd[q]))[:12]
        np.testing.assert_array_equal(I[q], o)
        np.testing.assert_array_equal(D[q], dd[q][o].astype(np.float32))


@pytest.mark.parametrize("fmt", ["faiss", "native"])
def test_save_load_roundtrip(tmp_path, golden_dir, fmt):
    z = load_case(golden_dir, "d96_m8_dsub12")
    ix = gpu_index(z)
    p = tmp_path / f"x.{fmt}"
    faiss.write_index(ix, p, fmt=fmt)
    iy = faiss.read_index(p, device=0)
    assert iy.ntotal == ix.ntotal and iy.nprobe == ix.nprobe
    for l in range(ix.nlist):
        np.testing.assert_array_equal(iy.invlists.get_ids(l), ix.invlists.get_ids(l))
        np.testing.assert_array_equal(iy.invlists.get_codes(l), ix.invlists.get_codes(l))
    D, I = iy.search(z["xq"], int(z["k"]))
    assert_same(D, I, z["or_D"], z["or_I"])


def test_index_factory_and_parameter_space(golden_dir):
    z = load_case(golden_dir, "d128_m16")
    ix = faiss.index_factory(128, "IVF64,PQ16")
    ix.set_trained(z["centroids"], z["codebook"])
    faiss.ParameterSpace().set_index_parameters(ix, "nprobe=8")
    assert ix.nprobe == 8
    assert ix.invlists.imbalance_factor() == 0.0


def test_errors_are_runtime_errors(golden_dir):
    z = load_case(golden_dir, "d128_m16")
    ix = gpu_index(z)
    with pytest.raises(RuntimeError):
        ix.search(z["xq"][:, :64], 10)
    with pytest.raises(RuntimeError):
        ix.search(z["xq"], 0)
    with pytest.raises(RuntimeError):
        ix.search(z["xq"], 1025)
    with pytest.raises(RuntimeError):
        faiss.IndexIVFPQ(None, 128, 64, 16, 8, device=0).search(z["xq"], 5)  # untrained
    with pytest.raises(RuntimeError):
        faiss.IndexIVFPQ(None, 100, 64, 16, 8, device=0)  # d % M != 0
