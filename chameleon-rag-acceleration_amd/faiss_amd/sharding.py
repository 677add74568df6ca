"""Multi-GPU IVF-PQ: inverted-list-range sharding with an RCCL exchange.

Replaces Faiss ``IndexShards`` (``bench_gpu_1bn.py:605-616``: query broadcast
to every GPU, per-shard top-k, host-side merge by CPU threads) and the host
``np.argsort`` shard merge (``bench_multi_cpu_performance_OSDI.py:203-218``).

One process per GPU (``torch.distributed``, backend ``nccl`` = RCCL on ROCm):

* GPU ``r`` stores and scans only the inverted lists ``[lo_r, hi_r)``; the
  ranges are contiguous and balanced by code bytes (lists are imbalanced,
  ``bench_polysemous_1bn.py:368``).
* Every rank holds the global query batch (``world`` slices of ``B`` queries,
  slice ``j`` owned by rank ``j``).  Rank ``j`` runs the coarse quantizer for
  its own slice only; one ``all_gather`` of the ``[B, nprobe]`` (list, dis0)
  arrays (``B * nprobe * 12`` bytes per rank, ~200 KB at C2) gives every rank
  the probes of the whole batch, and it scans its own lists for them
  (``search_preassigned``: the same pairs and dis0 as an unsharded search, so
  the result is bit-identical).  Per-rank coarse work stays flat in N; the T3
  tables (61 kFLOP per query) are built for the whole batch.
* One ``all_to_all`` sends slice ``j`` of every partial result to rank ``j``
  (``world * B * k * 12`` bytes per rank — latency-bound on xGMI), and each
  rank merges its ``world`` partial lists by (distance, label) on the GPU.

The exchange is written against plain ``torch.distributed`` so it runs under
``gloo`` on CPU tensors for the multi-process tests.
"""
from __future__ import annotations

import numpy as np


def balanced_list_ranges(list_sizes, world, code_size=1):
    """Contiguous list ranges [(lo, hi)] * world with near-equal code bytes.

    Greedy prefix cut: range r ends at the first list where the cumulative
    bytes reach (r + 1) / world of the total.  Every range is non-empty when
    nlist >= world.
    """
    sizes = np.asarray(list_sizes, dtype=np.int64) * int(code_size)
    nlist = sizes.shape[0]
    if world < 1 or world > nlist:
        raise ValueError("need 1 <= world <= nlist")
    csum = np.cumsum(sizes)
    total = csum[-1] if nlist else 0
    bounds = [0]
    for r in range(1, world):
        target = total * r / world
        cut = int(np.searchsorted(csum, target, side="left")) + 1
        cut = max(cut, bounds[-1] + 1)  # non-empty
        cut = min(cut, nlist - (world - r))  # leave one list per remaining rank
        bounds.append(cut)
    bounds.append(nlist)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def _coalesced(group, device):
    """One RCCL launch for the two collectives of an exchange (distances and labels):
    torch's coalescing manager around them when the group is an nccl (RCCL) group;
    a null context otherwise (gloo, the CPU tests)."""
    import contextlib

    import torch.distributed as dist

    if dist.get_backend(group) != "nccl":
        return contextlib.nullcontext()
    return dist.distributed_c10d._coalescing_manager(group=group, device=device)


def exchange_partials(Dp, Ip, world, group=None, force=False):
    """all_to_all of per-rank partial results.

    Dp, Ip: [world * B, k] partial top-k over this rank's lists for the global
    batch.  Returns (Ds, Is) of shape [world, B, k]: entry s holds rank s's
    partial for this rank's query slice.  One ``all_to_all_single`` per array:
    row block j of the input (slice j of the batch) goes to rank j, and the
    output's row block s comes from rank s (RCCL over xGMI on GPUs; gloo runs
    the same call on CPU tensors in the multi-process tests).  ``force``: run the
    collective even at world 1 (bench.py --shard-at-1: the RCCL calls and their
    communicator stream exist as they would at N > 1).
    """
    import torch
    import torch.distributed as dist

    n, k = Dp.shape
    B = n // world
    Ds = torch.empty((world, B, k), dtype=Dp.dtype, device=Dp.device)
    Is = torch.empty((world, B, k), dtype=Ip.dtype, device=Ip.device)
    if world == 1 and not force:
        Ds[0].copy_(Dp)
        Is[0].copy_(Ip)
        return Ds, Is
    Dp, Ip = Dp.contiguous(), Ip.contiguous()
    with _coalesced(group, Dp.device):
        dist.all_to_all_single(Ds.view(world * B, k), Dp, group=group)
        dist.all_to_all_single(Is.view(world * B, k), Ip, group=group)
    return Ds, Is


def all_gather_probes(Dq, Iq, world, group=None, force=False):
    """All-gather of the per-slice coarse results: [B, nprobe] -> [world * B, nprobe]
    (slice r from rank r), one ``all_gather_into_tensor`` per array (``force``: also
    at world 1, see exchange_partials)."""
    import torch
    import torch.distributed as dist

    if world == 1 and not force:
        return Dq, Iq
    outD = torch.empty((world * Dq.shape[0], Dq.shape[1]), dtype=Dq.dtype, device=Dq.device)
    outI = torch.empty((world * Iq.shape[0], Iq.shape[1]), dtype=Iq.dtype, device=Iq.device)
    Dq, Iq = Dq.contiguous(), Iq.contiguous()
    with _coalesced(group, Dq.device):
        dist.all_gather_into_tensor(outD, Dq, group=group)
        dist.all_gather_into_tensor(outI, Iq, group=group)
    return outD, outI


def exchange_and_gather(Dp, Ip, Dq, Iq, world, group=None, force=False):
    """One collective launch per shard step: the all_to_all of an earlier batch's
    partials (exchange_partials) and the all_gather of this batch's probes
    (all_gather_probes), issued together under one coalescing manager, so an RCCL
    group holds the CUs once per step instead of twice.  ``Dp``/``Ip`` may be None
    (no earlier batch pending).  Returns (Ds, Is, Dq_all, Iq_all); Ds/Is are None
    when Dp is.  Every rank must call it with the same pattern of None (the
    collectives are matched by order)."""
    import torch
    import torch.distributed as dist

    if world == 1 and not force:
        Ds = Is = None
        if Dp is not None:
            Ds, Is = Dp.unsqueeze(0).clone(), Ip.unsqueeze(0).clone()
        return Ds, Is, Dq, Iq
    outD = torch.empty((world * Dq.shape[0], Dq.shape[1]), dtype=Dq.dtype, device=Dq.device)
    outI = torch.empty((world * Iq.shape[0], Iq.shape[1]), dtype=Iq.dtype, device=Iq.device)
    Dq, Iq = Dq.contiguous(), Iq.contiguous()
    Ds = Is = None
    with _coalesced(group, Dq.device):
        if Dp is not None:
            n, k = Dp.shape
            B = n // world
            Ds = torch.empty((world, B, k), dtype=Dp.dtype, device=Dp.device)
            Is = torch.empty((world, B, k), dtype=Ip.dtype, device=Ip.device)
            Dp, Ip = Dp.contiguous(), Ip.contiguous()
            dist.all_to_all_single(Ds.view(world * B, k), Dp, group=group)
            dist.all_to_all_single(Is.view(world * B, k), Ip, group=group)
        dist.all_gather_into_tensor(outD, Dq, group=group)
        dist.all_gather_into_tensor(outI, Iq, group=group)
    return Ds, Is, outD, outI


def merge_partials_reference(Ds, Is):
    """Host merge of [S, n, k] sorted partials by (distance, label); -1 labels last.
    Test reference for the device merge (faiss_amd.merge_topk_device)."""
    Ds = np.asarray(Ds)
    Is = np.asarray(Is)
    S, n, k = Ds.shape
    D = np.empty((n, k), np.float32)
    I = np.empty((n, k), np.int64)
    big = np.iinfo(np.int64).max
    for q in range(n):
        dd = Ds[:, q].reshape(-1)
        ii = Is[:, q].reshape(-1)
        o = np.lexsort((np.where(ii < 0, big, ii), dd))[:k]
        D[q] = dd[o]
        I[q] = ii[o]
    return D, I


class ShardedSearch:
    """Per-rank driver of a list-range-sharded search.

    With ``coarse(x_slice) -> (Dq, Iq)`` and ``local_preassigned(xq_global, k,
    Iq, Dq) -> (Dp, Ip)`` (``IndexIVFPQ.coarse_device`` and
    ``search_preassigned_device`` in production) the coarse quantizer runs on
    this rank's query slice only and the probes are all-gathered; otherwise
    ``local_search(xq_global, k)`` runs the whole search of the global batch on
    this rank's lists.  ``merge(Ds, Is) -> (D, I)`` merges the exchanged
    partials (``faiss_amd.merge_topk_device`` in production).
    """

    def __init__(self, local_search, merge, world, group=None, coarse=None, local_preassigned=None):
        self.local_search = local_search
        self.merge = merge
        self.world = world
        self.group = group
        self.coarse = coarse
        self.local_preassigned = local_preassigned

    def partials(self, xq_global, k):
        """This rank's partial top-k [world * B, k] over its lists for the global batch."""
        if self.coarse is None or self.local_preassigned is None:
            return self.local_search(xq_global, k)
        import torch.distributed as dist

        rank = dist.get_rank(self.group) if self.world > 1 else 0
        B = xq_global.shape[0] // self.world
        Dq, Iq = self.coarse(xq_global[rank * B:(rank + 1) * B])
        Dq, Iq = all_gather_probes(Dq, Iq, self.world, self.group)
        return self.local_preassigned(xq_global, k, Iq, Dq)

    def search(self, xq_global, k):
        Dp, Ip = self.partials(xq_global, k)
        Ds, Is = exchange_partials(Dp, Ip, self.world, self.group)
        return self.merge(Ds, Is)
