"""Multi-process list-range sharding on CPU (gloo, world_size 2).

Each rank holds only its inverted-list range; the partial results of the
global batch are exchanged (all_to_all_single; gloo runs the same collectives) and merged by
(distance, label).  The sharded result must equal the unsharded oracle search.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from faiss_amd.sharding import balanced_list_ranges, merge_partials_reference


def test_balanced_list_ranges():
    sizes = np.array([5, 0, 100, 3, 3, 3, 50, 1, 0, 7])
    for world in (1, 2, 3, 5, 10):
        rg = balanced_list_ranges(sizes, world)
        assert rg[0][0] == 0 and rg[-1][1] == len(sizes)
        assert all(lo < hi for lo, hi in rg)
        assert all(rg[i][1] == rg[i + 1][0] for i in range(world - 1))
    rg = balanced_list_ranges(np.ones(1024), 8)
    assert [hi - lo for lo, hi in rg] == [128] * 8
    with pytest.raises(ValueError):
        balanced_list_ranges(np.ones(3), 4)


def test_merge_partials_reference_handles_padding():
    big = np.finfo(np.float32).max
    Ds = np.array([[[1, 3, big]], [[2, 3, 4]]], np.float32)
    Is = np.array([[[10, 30, -1]], [[20, 29, 40]]], np.int64)
    D, I = merge_partials_reference(Ds, Is)
    np.testing.assert_array_equal(I[0], [10, 20, 29])
    np.testing.assert_array_equal(D[0], [1, 2, 3])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, golden, out, slice_coarse=False):
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    sys.path.insert(0, os.path.join(repo, "chameleon-rag-acceleration_amd"))
    import torch
    import torch.distributed as dist

    from faiss_amd.sharding import ShardedSearch, balanced_list_ranges
    from oracle import oracle as O

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    z = dict(np.load(golden))
    d, M, nlist, k = int(z["d"]), int(z["M"]), int(z["nlist"]), int(z["k"])
    sizes = np.diff(z["list_off"])
    lo, hi = balanced_list_ranges(sizes, world, M)[rank]
    ox = O.OracleIVFPQ(d, nlist, M)
    ox.set_trained(z["centroids"], z["codebook"])
    list_no = np.repeat(np.arange(nlist, dtype=np.int64), sizes)
    keep = (list_no >= lo) & (list_no < hi)
    ox.add_preencoded(list_no[keep], z["codes"][keep], z["ids"][keep])
    ox.nprobe = int(z["nprobe"])

    def local(xq, kk):
        D, I = ox.search(xq.numpy(), kk)
        return torch.from_numpy(D), torch.from_numpy(I)

    def merge(Ds, Is):
        D, I = merge_partials_reference(Ds.numpy(), Is.numpy())
        return torch.from_numpy(D), torch.from_numpy(I)

    def coarse(xs):  # this rank's query slice only
        dis, lists = O.coarse_search(xs.numpy(), z["centroids"], ox.nprobe)
        return torch.from_numpy(dis), torch.from_numpy(lists)

    def local_pre(xq, kk, Iq, Dq):  # the gathered probes of the whole batch, this rank's lists
        D, I = ox.search_preassigned(xq.numpy(), kk, Iq.numpy(), Dq.numpy())
        return torch.from_numpy(D), torch.from_numpy(I)

    xq = torch.from_numpy(z["xq"])  # global batch: world slices
    ss = ShardedSearch(local, merge, world, coarse=coarse if slice_coarse else None,
                       local_preassigned=local_pre if slice_coarse else None)
    D, I = ss.search(xq, k)
    gD = [torch.empty_like(D) for _ in range(world)]
    gI = [torch.empty_like(I) for _ in range(world)]
    dist.all_gather(gD, D)
    dist.all_gather(gI, I)
    if rank == 0:
        np.savez(out, D=torch.cat(gD).numpy(), I=torch.cat(gI).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("slice_coarse", [False, True], ids=["global_coarse", "sliced_coarse_allgather"])
@pytest.mark.parametrize("case", ["d128_m16", "d96_m8_dsub12"])
def test_sharded_search_equals_unsharded(tmp_path, golden_dir, case, slice_coarse):
    """Both shard flows: every rank probing the whole batch, and each rank probing
    its own query slice with the (list, dis0) arrays all-gathered."""
    world = 2
    golden = os.path.join(golden_dir, f"ivfpq_{case}.npz")
    out = str(tmp_path / "res.npz")
    mp.spawn(_worker, args=(world, _free_port(), golden, out, slice_coarse), nprocs=world, join=True)
    r = np.load(out)
    z = np.load(golden)
    np.testing.assert_array_equal(r["I"], z["or_I"])
    np.testing.assert_array_equal(r["D"], z["or_D"])


def _collective_worker(rank, world, port, out):
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "chameleon-rag-acceleration_amd"))
    import torch
    import torch.distributed as dist

    from faiss_amd.sharding import all_gather_probes, exchange_and_gather, exchange_partials

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    B, k, np_ = 5, 3, 4
    g = torch.Generator().manual_seed(rank)
    Dp = torch.rand((world * B, k), generator=g)
    Ip = torch.randint(0, 1 << 40, (world * B, k), generator=g)
    Ds, Is = exchange_partials(Dp, Ip, world)
    # reference: gather every rank's whole partial array, then take this rank's slice of each
    gD = [torch.empty_like(Dp) for _ in range(world)]
    gI = [torch.empty_like(Ip) for _ in range(world)]
    dist.all_gather(gD, Dp)
    dist.all_gather(gI, Ip)
    ok = all(torch.equal(Ds[s], gD[s][rank * B:(rank + 1) * B]) and torch.equal(Is[s], gI[s][rank * B:(rank + 1) * B])
             for s in range(world))
    Dq = torch.rand((B, np_), generator=g)
    Iq = torch.randint(0, 1024, (B, np_), generator=g)
    aD, aI = all_gather_probes(Dq, Iq, world)
    hD = [torch.empty_like(Dq) for _ in range(world)]
    hI = [torch.empty_like(Iq) for _ in range(world)]
    dist.all_gather(hD, Dq)
    dist.all_gather(hI, Iq)
    ok = ok and torch.equal(aD, torch.cat(hD)) and torch.equal(aI, torch.cat(hI))
    # bench.py with batches in flight: one process group per in-flight stream, used
    # alternately; every group gives the same slices as the default one
    groups = [dist.new_group(list(range(world))) for _ in range(2)]
    for step in range(4):
        grp = groups[step % 2]
        Ds2, Is2 = exchange_partials(Dp, Ip, world, grp)
        aD2, aI2 = all_gather_probes(Dq, Iq, world, grp)
        ok = ok and torch.equal(Ds2, Ds) and torch.equal(Is2, Is) and torch.equal(aD2, aD) and torch.equal(aI2, aI)
    # bench.py's fused step exchange: the earlier batch's all_to_all and this batch's
    # all_gather in one call (and the first step, with no earlier batch)
    Ds3, Is3, aD3, aI3 = exchange_and_gather(Dp, Ip, Dq, Iq, world, groups[0])
    ok = ok and torch.equal(Ds3, Ds) and torch.equal(Is3, Is) and torch.equal(aD3, aD) and torch.equal(aI3, aI)
    n3 = exchange_and_gather(None, None, Dq, Iq, world)
    ok = ok and n3[0] is None and n3[1] is None and torch.equal(n3[2], aD) and torch.equal(n3[3], aI)
    flags = [torch.zeros(1) for _ in range(world)]
    dist.all_gather(flags, torch.tensor([1.0 if ok else 0.0]))
    if rank == 0:
        np.save(out, np.array([float(f) for f in flags]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_exchange_collectives_slicing(tmp_path, world):
    """The collectives bench.py's shard step runs over RCCL (all_to_all_single of
    the partials, all_gather_into_tensor of the probes; on the default group and on
    the per-stream groups of batches in flight), executed here under gloo:
    rank r receives slice r of every rank's partials in rank order, and the
    probes of slice s come from rank s -- the layout of a gather-then-slice
    reference."""
    out = str(tmp_path / "ok.npy")
    mp.spawn(_collective_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    assert np.load(out).tolist() == [1.0] * world
