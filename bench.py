#!/usr/bin/env python3
"""bench.py — IVF-PQ search throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): SIFT1M-shaped synthetic
data (d=128, 1M base, 100k train, 10,240 queries; clustered, integer-valued
float32), IndexIVFPQ "IVF1024,PQ16" (8-bit codes) trained on the GPU, nprobe=16,
k=10, query batch 1024.  One *step* = one whole search of one 1024-query batch
(coarse probe + inner-product table + fused LUT/scan/top-k) with the queries
already resident in HBM.

N > 1 (one process per GPU, torch.distributed over RCCL; weak scaling, 1024
queries per GPU per step).  Default ``--mode shard``, the north_star design: the
index is split by inverted-list range, each rank runs the coarse quantizer on its
own 1024-query slice, an all_gather shares the (list, dis0) probe arrays, every
rank scans its lists for the whole batch (search_preassigned) and an all_to_all
returns each query slice's partials to its owner, which merges them on the GPU.
Beside it (``extra.replicas``) the same ranks also time query-sharded replicas
(each rank holds the whole index and searches its own batches, no collective on
the data path) and check that the sharded results equal the replica's, bit for
bit.  ``--mode replicas`` makes the replicas the value.

Prints ONE JSON line on rank 0 (contract in the task statement), with
``roofline`` (the scan kernel's algorithmic code bytes / its HIP-event-timed
duration against 8 TB/s) and ``cpu_baseline`` (the oracle's Faiss-1.7.1-order
C restatement, OpenMP over queries, on a bounded sample of the same queries).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "chameleon-rag-acceleration_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def lib_sha256():
    import hashlib

    from faiss_amd import _lib

    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--batch", type=int, default=1024)
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--nprobe", type=int, default=16)
    p.add_argument("--nlist", type=int, default=1024)
    p.add_argument("--M", type=int, default=16)
    p.add_argument("--d", type=int, default=128)
    p.add_argument("--nb", type=int, default=1_000_000)
    p.add_argument("--nt", type=int, default=100_000)
    p.add_argument("--nbatches", type=int, default=10)
    p.add_argument("--niter", type=int, default=25)
    p.add_argument("--centres", type=int, default=200_000,
                   help="Gaussian centres of the synthetic generator (200k: the recall curve tracks SIFT1M's; "
                        "rounds 1-2 used 10k)")
    p.add_argument("--mode", choices=["shard", "replicas"], default="shard")
    p.add_argument("--shard-at-1", action="store_true",
                   help="run the list-range shard flow at WORLD_SIZE=1 too, with a real nccl (RCCL) process group of "
                        "one rank: every collective of the N > 1 step is a real RCCL call and its communicator stream "
                        "exists (the stream topology the scaling run uses, measured on one GPU)")
    p.add_argument("--stream-priority", choices=["normal", "high"], default="normal",
                   help="priority of the in-flight compute streams (high: ahead of RCCL's communicator stream)")
    p.add_argument("--rccl-priority", choices=["normal", "high"], default="normal",
                   help="shard flow: priority of RCCL's communicator stream (high: its collective kernels are "
                        "dispatched ahead of the compute streams' pending workgroups)")
    p.add_argument("--comms", choices=["one", "per-stream"], default="one",
                   help="shard flow: one communicator for every in-flight stream (default; the loop issues each "
                        "batch's all_to_all after the next batch's all_gather, so the communicator's stream never "
                        "holds a batch behind another's scan) or one per in-flight stream")
    p.add_argument("--no-peak", action="store_true", help="skip the HBM stream-copy peak measurement")
    p.add_argument("--cpu-sample", type=int, default=10240, help="queries in the CPU-baseline sample")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline time budget (repetitions)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--event-every", type=int, default=5,
                   help="record the list-scan HIP events on every N-th timed step")
    p.add_argument("--no-recall", action="store_true")
    p.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "r06_scan_pmc.json"),
                   help="counter-measured HBM bytes of the scan kernel; used only if its lib_sha256 matches "
                        "the library loaded now")
    p.add_argument("--no-extra", action="store_true", help="skip the k=100 and host-path search() rates")
    p.add_argument("--inflight", type=int, default=None,
                   help="batches in flight on that many HIP streams (step s on stream s %% N, each with its own "
                        "workspace; > 1 turns the index's batches-in-flight mode on so that consecutive batches "
                        "overlap, DESIGN.md section 4); 1 = one batch at a time on one stream (also measured beside "
                        "the value as ms_per_step_serial).  Default: 2, or 3 in the shard flow (three compute "
                        "streams + one RCCL communicator = the box's four hardware queues); DESIGN.md section 5 "
                        "has the depth A/Bs (plain: 0.109 / 0.123 / 0.110 ms with 2 / 3 / 4; shard flow at world "
                        "size 1: noisy, 0.14-0.20 ms with 3 and 0.17-0.19 with 2; one-GPU emulation at N = 2-8: "
                        "3 at or below 2)")
    return p.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    shard = args.mode == "shard" and (world > 1 or args.shard_at_1)
    if world > 1 or shard:
        if world == 1:  # --shard-at-1: a one-rank RCCL group on the loopback rendezvous
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(29500 + os.getpid() % 2000))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if args.rccl_priority == "high":
            opts = dist.ProcessGroupNCCL.Options()
            opts.is_high_priority_stream = True
            dist.init_process_group("nccl", device_id=dev, pg_options=opts)
        else:
            dist.init_process_group("nccl", device_id=dev)

    import faiss_amd as faiss
    from faiss_amd import datasets
    from faiss_amd.sharding import balanced_list_ranges, exchange_and_gather, exchange_partials

    t_setup = time.time()
    B = args.batch
    Bg = B * world if shard else B  # queries per step on each rank
    log(f"rank {rank}/{world} generating data nb={args.nb} nt={args.nt}")
    gen = dict(n_centres=args.centres)
    xt = datasets.synthetic_sift_like(args.nt, args.d, seed=4321, **gen)
    xb = datasets.synthetic_sift_like(args.nb, args.d, seed=1234, **gen)
    nq_total = args.nbatches * Bg
    xq = datasets.synthetic_sift_like(nq_total, args.d, seed=123 + (0 if shard else rank), **gen)

    ix = faiss.index_factory(args.d, f"IVF{args.nlist},PQ{args.M}", device=local_rank)
    ix.niter_coarse = ix.niter_pq = args.niter
    t0 = time.time()
    ix.train(xt)
    log(f"trained in {time.time() - t0:.1f}s")
    lo, hi = 0, args.nlist
    if shard:
        # balance list ranges by code bytes: assign the base set once (top-1)
        ix.nprobe = 1
        sizes = np.zeros(args.nlist, np.int64)
        for i0 in range(0, args.nb, 1 << 18):
            xbd = torch.from_numpy(xb[i0:i0 + (1 << 18)]).to(dev)
            _, Iq = ix.coarse_device(xbd)
            sizes += np.bincount(Iq[:, 0].cpu().numpy(), minlength=args.nlist)
        lo, hi = balanced_list_ranges(sizes, world, args.M)[rank]
        ix.set_list_range(lo, hi)
    t0 = time.time()
    ix.add(xb)
    log(f"added {ix.ntotal} vectors (lists [{lo},{hi})) in {time.time() - t0:.1f}s")
    ix.nprobe = args.nprobe
    list_sizes = ix.invlists.list_sizes()

    xq_dev = torch.from_numpy(xq).to(dev).view(args.nbatches, Bg, args.d)
    k = args.k
    inflight = max(1, args.inflight if args.inflight is not None else (3 if shard else 2))
    ix.inflight = inflight > 1
    # Streams of the timed region, per process: `inflight` compute
    # streams, plus, sharded, the communicator streams of RCCL -- one communicator (the
    # default group) for every in-flight stream, or (--comms per-stream) one each.  No
    # side streams: T3 of the global batch rides in the coarse launch of the batch's own
    # stream (coarse_tables_device).
    if shard:
        groups = ([dist.new_group(list(range(world))) for _ in range(inflight)] if args.comms == "per-stream"
                  else [dist.group.WORLD] * inflight)
    else:
        groups = None
    streams = [torch.cuda.Stream(dev, priority=-1 if args.stream_priority == "high" else 0) for _ in range(inflight)]
    Dbufs = [torch.empty((Bg, k), dtype=torch.float32, device=dev) for _ in range(inflight)]
    Ibufs = [torch.empty((Bg, k), dtype=torch.int64, device=dev) for _ in range(inflight)]
    Dbuf, Ibuf = Dbufs[0], Ibufs[0]

    # algorithmic bytes: code_size x codes of every probed list in this
    # rank's range, per batch; the list-scan kernel covers all of them
    bytes_alg = []
    for b in range(args.nbatches):
        _, Iq = ix.coarse_device(xq_dev[b])
        Iq = Iq.cpu().numpy()
        sz = np.where(Iq >= 0, list_sizes[np.maximum(Iq, 0)], 0)  # lists outside [lo, hi) have size 0 here
        bytes_alg.append(int(sz.sum()) * args.M)
    bytes_lists = bytes_alg

    merged = {}
    pend = [None] * inflight  # sharded: the batch whose partials stream j has not exchanged yet

    def back(j):
        # the partials of stream j's pending batch to their owners, merged on the GPU
        # (the drain at the end of a timed region; in the loop the exchange rides with
        # the next batch's all_gather, below)
        b, Dp, Ip = pend[j]
        pend[j] = None
        with torch.cuda.stream(streams[j]):
            Ds, Is = exchange_partials(Dp, Ip, world, groups[j], force=True)
            merged[b] = faiss.merge_topk_device(Ds, Is)

    def step(b, j=0):
        if shard:
            # stream j: coarse of this rank's slice + T3 of the global batch (one
            # launch); ONE collective launch that returns stream j's previous batch's
            # partials to their owners and all-gathers this batch's probes; the previous
            # batch's merge; this rank's lists scanned for the whole batch.  On a shared
            # communicator every rank issues the same sequence, and batch s waits only
            # for batch s - inflight's scan
            prev = pend[j]
            pend[j] = None
            xg = xq_dev[b]
            with torch.cuda.stream(streams[j]):
                Dq_s, Iq_s, tok = ix.coarse_tables_device(xg[rank * B:(rank + 1) * B], xg)
                Ds, Is, Dq, Iq = exchange_and_gather(prev[1] if prev else None, prev[2] if prev else None,
                                                     Dq_s, Iq_s, world, groups[j], force=True)
                if prev is not None:
                    merged[prev[0]] = faiss.merge_topk_device(Ds, Is)
                Dp, Ip = ix.search_preassigned_device(xg, k, Iq, Dq, Dbufs[j], Ibufs[j], tables=tok)
            pend[j] = (b, Dp, Ip)
        else:  # stream j of the in-flight set, with its own output buffers
            ix.search_device(xq_dev[b], k, Dbufs[j], Ibufs[j], stream=streams[j].cuda_stream)

    def drain():
        for j in range(inflight):
            if pend[j] is not None:
                back(j)

    def serial_step(b):  # one batch at a time on stream 0
        step(b, 0)
        drain()

    for j in range(inflight):  # setup: each in-flight stream's workspace allocated, whatever --warmup is
        step(j % args.nbatches, j)
    drain()
    torch.cuda.synchronize()
    for w in range(args.warmup):
        step(w % args.nbatches, w % inflight)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()

    # the box's measured HBM peak (STREAM copy and a read sweep, 2 GiB each, best of 10),
    # beside the nominal 8 TB/s
    peak_measured = None
    if not args.no_peak:
        try:
            import ctypes

            hl = ctypes.CDLL(os.path.join(REPO, "chameleon-rag-acceleration_amd", "lib", "libhbmstream.so"))
            nbytes = 2 << 30
            src = torch.empty(nbytes // 4, dtype=torch.int32, device=dev).random_(0, 1 << 30)
            dst = torch.empty_like(src)
            sink = torch.empty(1 << 22, dtype=torch.int32, device=dev)
            cms, rms = ctypes.c_float(0), ctypes.c_float(0)
            rc = hl.hbm_stream_measure(ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(dst.data_ptr()),
                                       ctypes.c_int64(nbytes), ctypes.c_void_p(sink.data_ptr()),
                                       ctypes.c_int64(sink.numel() * 4), 10,
                                       ctypes.c_void_p(torch.cuda.current_stream().cuda_stream),
                                       ctypes.byref(cms), ctypes.byref(rms))
            if rc == 0:
                peak_measured = {"copy_GBps": 2 * nbytes / (cms.value * 1e-3) / 1e9,
                                 "read_GBps": nbytes / (rms.value * 1e-3) / 1e9,
                                 "copy_ms": cms.value, "read_ms": rms.value, "bytes": nbytes,
                                 "kernel": "csrc/hbm_stream.hip (16 B per lane, nontemporal, 8 workgroups per CU, "
                                           "best of 10; copy counts read + written bytes)"}
            del src, dst, sink
            torch.cuda.synchronize()
        except OSError as e:
            log(f"hbm peak not measured: {e}")
    log(f"setup {time.time() - t_setup:.1f}s; timing {args.steps} steps")

    # timed region: HIP events around the list-scan kernel only, on every
    # --event-every-th step (each recorded event costs ~6 us of stream time; the
    # full stage split is measured in a separate pass below)
    rs0 = ix.repair_stats()  # (waits for in-flight searches)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        ix.set_timing(s % args.event_every == 0, lists_only=True)
        step(s % args.nbatches, s % inflight)
    drain()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    rs1 = ix.repair_stats()  # stale partial lists the merge repaired in the timed region: must be 0
    ix.set_timing(False)
    stages = ix.get_timing()
    # the same steps one batch at a time on one stream (reported beside the value)
    serial_ms, stages_serial = None, None
    if inflight > 1:
        ix.inflight = False  # one batch at a time: the handle's serial mode (full scan grid)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for s in range(args.steps):
            ix.set_timing(s % args.event_every == 0, lists_only=True)
            serial_step(s % args.nbatches)
        torch.cuda.synchronize()
        serial_ms = (time.perf_counter() - t1) * 1000.0 / args.steps
        ix.set_timing(False)
        stages_serial = ix.get_timing()
    # stage breakdown (untimed pass, one stream, every stage bracketed by events)
    ix.set_timing(True)
    for s in range(args.steps):
        serial_step(s % args.nbatches)
    torch.cuda.synchronize()
    ix.set_timing(False)
    stage_split = ix.get_timing()
    ix.inflight = inflight > 1

    # extra rates (rank 0 view, untimed by the contract): k = 100 (the reference's
    # profiling K) on the device path, and the host-buffer search() (PCIe included)
    extra = {}
    if not args.no_extra and not shard:
        n_ex = max(5, min(50, args.steps))
        D100 = torch.empty((Bg, 100), dtype=torch.float32, device=dev)
        I100 = torch.empty((Bg, 100), dtype=torch.int64, device=dev)
        D100 = [D100] + [torch.empty_like(D100) for _ in range(inflight - 1)]
        I100 = [I100] + [torch.empty_like(I100) for _ in range(inflight - 1)]
        for j in range(inflight):
            ix.search_device(xq_dev[j % args.nbatches], 100, D100[j], I100[j], stream=streams[j].cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(n_ex):  # k = 100 with the same batches in flight as the value
            j = s % inflight
            ix.search_device(xq_dev[s % args.nbatches], 100, D100[j], I100[j], stream=streams[j].cuda_stream)
        torch.cuda.synchronize()
        extra["k100_queries_per_s"] = n_ex * Bg / (time.perf_counter() - t0)
        ix.inflight = False
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(n_ex):
            ix.search_device(xq_dev[s % args.nbatches], 100, D100[0], I100[0], stream=streams[0].cuda_stream)
        torch.cuda.synchronize()
        extra["k100_queries_per_s_serial"] = n_ex * Bg / (time.perf_counter() - t0)
        ix.inflight = inflight > 1
        xq_host = [np.ascontiguousarray(xq[b * Bg:(b + 1) * Bg]) for b in range(args.nbatches)]
        ix.search(xq_host[0], k)
        t0 = time.perf_counter()
        for s in range(n_ex):
            ix.search(xq_host[s % args.nbatches], k)
        extra["host_search_queries_per_s"] = n_ex * Bg / (time.perf_counter() - t0)
        extra["note"] = (f"{n_ex} batches each; k100 = search_device with k=100 and {inflight} batches in flight "
                         f"(k100_serial: one at a time on one stream); host_search = search() on numpy "
                         f"queries (H2D copy, search, D2H copy; synchronous)")
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # (a full replica of the index on every rank: only where it fits beside the shard)
    rep_fits = args.nb * (args.M + 8) < (32 << 30)
    if shard and not args.no_extra and rep_fits:
        # Beside the sharded value: query-sharded replicas (every rank the whole index,
        # its own slice of each global batch) on the same ranks, and the sharded results
        # checked against the replica's search of the same queries (bit for bit).
        ix_rep = faiss.IndexIVFPQ(None, args.d, args.nlist, args.M, 8, device=local_rank)
        ix_rep.set_trained(ix.centroids(), ix.codebook())
        ix_rep.add(xb)
        ix_rep.nprobe = args.nprobe
        mine = [xq_dev[b][rank * B:(rank + 1) * B].contiguous() for b in range(args.nbatches)]
        agree, rows = 0, 0
        for b in range(args.nbatches):
            serial_step(b)
            Dr, Ir = ix_rep.search_device(mine[b], k)
            torch.cuda.synchronize()
            Dm, Im = merged[b]
            agree += int(((Im == Ir).all(dim=1) & (Dm == Dr).all(dim=1)).sum().item())
            rows += B
        ix_rep.inflight = inflight > 1
        for b in range(max(args.warmup, inflight)):
            j = b % inflight
            ix_rep.search_device(mine[b % args.nbatches], k, Dbufs[j][:B], Ibufs[j][:B], stream=streams[j].cuda_stream)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(args.steps):  # the same batches in flight as the sharded value
            j = s % inflight
            ix_rep.search_device(mine[s % args.nbatches], k, Dbufs[j][:B], Ibufs[j][:B], stream=streams[j].cuda_stream)
        torch.cuda.synchronize()
        dist.barrier()
        tr = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
        dist.all_reduce(tr, op=dist.ReduceOp.MAX)
        ag = torch.tensor([agree, rows], dtype=torch.int64, device=dev)
        dist.all_reduce(ag)
        extra["replicas"] = {"queries_per_s": args.steps * B * world / float(tr.item()),
                             "ms_per_step": float(tr.item()) * 1e3 / args.steps,
                             "note": "each rank the whole index and its own 1024 queries per step, no collective"}
        extra["shard_vs_replica_rows_identical"] = f"{int(ag[0].item())} / {int(ag[1].item())}"
        del ix_rep

    queries = args.steps * B * world  # all ranks together
    qps = queries / elapsed
    ms_per_step = elapsed * 1000.0 / args.steps
    scan_ms, scan_n = stage_split["scan"]
    scan_avg_ms = scan_ms / max(scan_n, 1)
    lists_ms, lists_n = stages["lists"]
    bytes_per_step = sum(bytes_alg[s % args.nbatches] for s in range(args.steps)) / args.steps
    kernel = (f"k_scan_lean<{args.M},...> (list-major LUT + PQ scan + row-packed top-k, every probe)"
              if k <= 16 and args.M <= 16 else
              f"k_scan_lists<{args.M},...> (list-major LUT + PQ scan + top-k, every probe)")
    avg_launch_ms = lists_ms / max(lists_n, 1)
    timed = [s for s in range(args.steps) if s % args.event_every == 0]  # the steps with events
    bytes_per_launch = sum(bytes_lists[s % args.nbatches] for s in timed) / len(timed)
    achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9
    overlapped = None
    measured_on = "the timed region (one batch at a time)"
    if stages_serial and stages_serial["lists"][1] > 0:
        # Batches in flight: in the timed region a scan launch shares the chip with the
        # next batch's coarse step and scan start, so its event span is not the kernel's
        # own duration.  The roofline is taken from the same steps run one batch at a
        # time right after the timed region (ms_per_step_serial); the overlapped span is
        # reported beside it.
        overlapped = {"avg_launch_ms": avg_launch_ms, "achieved": achieved, "frac": achieved / HBM_PEAK_GBPS,
                      "note": f"scan-kernel event span in the timed region, {inflight} batches in flight"}
        avg_launch_ms = stages_serial["lists"][0] / stages_serial["lists"][1]
        achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9
        measured_on = ("the timed region's steps run again one batch at a time on one stream, right after it "
                       "(HIP events around each scan launch)")

    # ---------------------------------------------------------- recall (rank 0)
    recall = None
    cpu_baseline = None
    if rank == 0 and not args.no_recall:
        log("recall: exact float64 ground truth on the GPU")
        allI = []
        for b in range(args.nbatches):
            if shard:
                continue
            D, I = ix.search_device(xq_dev[b], k)
            allI.append(I.cpu().numpy())
        if allI:
            I_gpu = np.concatenate(allI)
            xb64 = torch.from_numpy(xb).to(dev, torch.float64)
            nb2 = (xb64 * xb64).sum(1)
            gt = []
            for i0 in range(0, I_gpu.shape[0], 256):
                q = torch.from_numpy(xq[i0:i0 + 256]).to(dev, torch.float64)
                dd = (q * q).sum(1, keepdim=True) + nb2[None, :] - 2.0 * (q @ xb64.T)
                gt.append(torch.topk(dd, k, dim=1, largest=False).indices.cpu().numpy())
            gt = np.concatenate(gt)
            del xb64, nb2
            r1 = datasets.recall_1_at(I_gpu, gt, (1, k))
            recall = {"R1@1": r1.get(1), f"R1@{k}": r1.get(k), f"R@{k}": datasets.recall_at_k(I_gpu, gt, k),
                      "queries": int(I_gpu.shape[0]), "gt": "exact float64 brute force"}

        if world == 1 and not args.no_cpu_baseline:
            from oracle import oracle as O

            log("cpu baseline: oracle on a bounded sample")
            ox = O.OracleIVFPQ(args.d, args.nlist, args.M)
            ox.set_trained(ix.centroids(), ix.codebook())
            for l in range(args.nlist):
                ox.list_ids[l] = ix.invlists.get_ids(l)
                ox.list_codes[l] = ix.invlists.get_codes(l).reshape(-1, args.M)
            ox.ntotal = ix.ntotal
            ox.nprobe = args.nprobe
            ns = min(args.cpu_sample, nq_total)
            # This process's share of the host: the GPU pool gives each GPU's jobs 16 host
            # cores and sets OMP_NUM_THREADS=16 on the box for it ("size worker pools to the
            # box's CPU share (16 for one GPU)"; os.sched_getaffinity there lists the whole
            # machine, which other GPUs' jobs share), so the oracle runs OMP_NUM_THREADS
            # threads when set, else every core of the affinity set (e.g. this container).
            affinity = len(os.sched_getaffinity(0))
            omp = os.environ.get("OMP_NUM_THREADS")
            threads = min(int(omp or 0) or affinity, affinity)

            def cpu_rate(nprobe_c):
                ox.nprobe = nprobe_c
                ox.search(xq[:64], k, threads)  # warm
                rates, tc, Ic = [], 0.0, None
                while len(rates) < 5 or (tc < args.cpu_seconds and len(rates) < 200):  # bounded: ~cpu_seconds
                    t0 = time.perf_counter()
                    _, Ic = ox.search(xq[:ns], k, threads)
                    dt = time.perf_counter() - t0
                    rates.append(ns / dt)
                    tc += dt
                return float(np.median(rates)), len(rates), tc, Ic

            rate, nrep, tc, Ic = cpu_rate(args.nprobe)
            agree = None
            if not shard:
                Ig = np.concatenate([ix.search(xq[i0:i0 + B], k)[1] for i0 in range(0, ns, B)])
                agree = float((Ig == Ic).mean())
            cpu_baseline = {"value": rate, "unit": "queries/s", "cores": threads, "kind": "port",
                            "cpu_model": cpu_model(), "cores_in_affinity": affinity,
                            "omp_num_threads_env": omp,
                            "cores_note": "the GPU pool's per-GPU host share is 16 cores, exported as "
                                          "OMP_NUM_THREADS=16 on the box (its rule: size worker pools to that "
                                          "share); without OMP_NUM_THREADS every core of the affinity set runs",
                            "sample": f"{ns} of the same queries (batch {B}), k={k}, nprobe={args.nprobe}, same "
                                      f"trained index; oracle/ivfpq_oracle.c (Faiss-1.7.1 order, scalar C, "
                                      f"OpenMP over queries); median of {nrep} repetitions, {tc:.1f}s total",
                            "gpu_id_agreement": agree}
            # BASELINE.json configs[0] (C1): the same index searched on the CPU at nprobe 8
            # (the reference publishes 0.164 ms/query and R1@10 0.8317 on SIFT1M,
            # Faiss_experiments/README.md:271), beside the GPU rate at nprobe 8
            rate8, nrep8, tc8, I8 = cpu_rate(8)
            c1 = {"cpu_queries_per_s": rate8, "cpu_ms_per_query_per_core": threads * 1e3 / rate8,
                  "cores": threads, "repetitions": nrep8, "seconds": round(tc8, 1),
                  "reference_sift1m": {"ms_per_query": 0.164, "R1@10": 0.8317}}
            if not shard:
                ix.nprobe = 8
                xd8 = xq_dev[0]
                ix.search_device(xd8, k, Dbuf, Ibuf)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for s in range(args.steps):
                    ix.search_device(xq_dev[s % args.nbatches], k, Dbuf, Ibuf)
                torch.cuda.synchronize()
                c1["gpu_queries_per_s"] = args.steps * B / (time.perf_counter() - t0)
                ix.nprobe = args.nprobe
                if recall is not None:
                    c1["R1@10_cpu_sample"] = datasets.recall_1_at(I8, gt[:ns], (1, k)).get(k)
            cpu_baseline["c1_nprobe8"] = c1

    traffic = None
    traffic_src = "no counter file"
    config_key = (f"nb{args.nb}-d{args.d}-IVF{args.nlist}-PQ{args.M}-np{args.nprobe}-k{k}-B{B}-w{world}-"
                  f"{args.mode if world > 1 else ('shard-at-1' if shard else 'single')}"
                  f"-c{args.centres}")
    sha = lib_sha256()
    from faiss_amd import _lib

    ksha = _lib.kernel_source_sha256()
    if os.path.exists(args.pmc_json):
        try:
            pm = json.load(open(args.pmc_json))
            if pm.get("config_key") != config_key:
                traffic_src = "counter file is for another config"
            elif pm.get("kernel_src_sha256") != ksha and pm.get("lib_sha256") != sha:
                traffic_src = "counter file is stale (measured on another build of the kernels)"
            else:
                traffic = pm.get("hbm_bytes_per_launch")
                traffic_src = os.path.relpath(args.pmc_json, REPO)
        except Exception as e:  # malformed file: report, never guess
            traffic_src = f"unreadable counter file: {e}"

    if rank == 0:
        out = {
            "metric": "queries/sec + recall@10, SIFT1M IVF-PQ (nlist=1024, M=16, nprobe=16)",
            "value": qps,
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "ms_per_step_serial": serial_ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": f"synthetic (SIFT1M-shaped clustered integer-valued float32, {args.centres} centres, sigma 16, "
                    "seeds base 1234 / train 4321 / queries 123); index trained on the GPU",
            "config": {
                "workload": f"IVF{args.nlist},PQ{args.M}x8 search, d={args.d}, nb={args.nb}, nprobe={args.nprobe}, "
                            f"k={k}, batch={B} queries per GPU per step",
                "parallelism": (f"list-range shards x{world} + RCCL all_gather / all_to_all ({args.comms} "
                                f"communicator{'s' if args.comms == 'per-stream' else ''})" if shard
                                else f"replicas x{world}" if world > 1 else "single GPU"),
                "global_batch": B * world,
                "inflight": inflight,
                "key": config_key,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "peak_measured": peak_measured["copy_GBps"] if peak_measured else None,
                "frac_measured": achieved / peak_measured["copy_GBps"] if peak_measured else None,
                "peak_measured_detail": peak_measured,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "lib_sha256": sha,
                "kernel_src_sha256": ksha,
                "kernel": kernel,
                "alg_bytes_per_launch": bytes_per_launch,
                "avg_launch_ms": avg_launch_ms,
                "measured_on": measured_on,
                "scan_stage": {"alg_bytes": bytes_per_step, "avg_ms": scan_avg_ms,
                               "achieved": bytes_per_step / (scan_avg_ms * 1e-3) / 1e9},
                "overlapped": overlapped,
                "end_to_end": {"alg_bytes": bytes_per_step, "ms_per_step": ms_per_step,
                               "achieved": bytes_per_step / (ms_per_step * 1e-3) / 1e9 if world == 1 else None},
            },
            "repairs": rs1[1] - rs0[1],
            "stale_reads": rs1[0] - rs0[0],
            "stages_ms_per_step": {s: v[0] / max(v[1], 1) for s, v in stage_split.items()},
            "recall": recall,
            "cpu_baseline": cpu_baseline,
            "extra": extra or None,
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
