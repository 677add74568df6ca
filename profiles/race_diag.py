#!/usr/bin/env python3
"""Batches-in-flight mismatch hunt (tests/test_gpu_parity.py
test_batches_in_flight_on_round_robin_streams scenario): the rr_index index
(IVF256,PQ8, d 64, nprobe 12), 24 batches of 256 queries issued round robin on
several streams with the handle's inflight mode on, compared with each batch
searched alone.  Per (k, streams, round): mismatching batches / rows, whether
the bad rows hold sentinel labels or non-finite keys, and the merge kernels'
index-check count.  Round 0 of each configuration is the first use of the
workspaces at that k (buffers grow there); later rounds reuse them.
Prints one JSON line per configuration, with the library's stale-entry counters
(repair_stats, cumulative over the configurations) and its first logged events
(repair_log).  r05: partial lists are tagged records; a stale entry is detected and
its probe rescanned by the merge, so "bad_batches" must now be 0."""
import json
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "chameleon-rag-acceleration_amd"))


def main():
    import numpy as np
    import torch

    import faiss_amd as faiss
    from faiss_amd import _lib, datasets

    configs = [(100, 3), (100, 2), (10, 3), (100, 4)]
    if len(sys.argv) > 1:
        configs = [tuple(int(v) for v in c.split(",")) for c in sys.argv[1:]]
    # (k, streams[, hog]): hog = 1 keeps a 512 MB device-to-device copy loop running on
    # a side stream (not the library's) while the batches run, with inflight off for
    # a single stream -- memory latency under load without batch overlap; hog = 2: a
    # coarse_device + preassigned search on batch 5's stream before it (the test's mix)
    rounds = int(os.environ.get("RACE_ROUNDS", "8"))
    xt = datasets.synthetic_sift_like(20_000, 64, seed=4321, n_centres=20_000)
    xb = datasets.synthetic_sift_like(100_000, 64, seed=1234, n_centres=20_000)
    xq = datasets.synthetic_sift_like(24 * 256, 64, seed=123, n_centres=20_000)
    ix = faiss.index_factory(64, "IVF256,PQ8", device=0)
    ix.niter_coarse = ix.niter_pq = 8
    ix.train(xt)
    ix.add(xb)
    ix.nprobe = 12
    nb = 24
    xd = torch.from_numpy(xq).cuda().view(nb, 256, 64)
    torch.cuda.synchronize()
    refs = {}
    for k in sorted({c[0] for c in configs}):
        ref = []
        for b in range(nb):
            D, I = ix.search_device(xd[b], k)
            torch.cuda.synchronize()
            ref.append((D.cpu().numpy(), I.cpu().numpy()))
        refs[k] = ref
    # coarse references (modes 3 and 4): the probes of every batch, searched alone
    cref = []
    for b in range(nb):
        Dq, Iq = ix.coarse_device(xd[b])
        torch.cuda.synchronize()
        cref.append((Dq.clone(), Iq.clone()))
    big = np.iinfo(np.int64).max
    hog_a = torch.empty(1 << 27, device="cuda")
    hog_b = torch.empty_like(hog_a)
    side = torch.cuda.Stream()
    for cfg in configs:
        k, nst = cfg[0], cfg[1]
        hog = len(cfg) > 2 and cfg[2] == 1
        mix = len(cfg) > 2 and cfg[2] == 2
        coarse_only = len(cfg) > 2 and cfg[2] == 3  # mode 3: coarse_device only, vs its reference
        pre_only = len(cfg) > 2 and cfg[2] == 4     # mode 4: search_preassigned_device with the reference probes
        t0 = time.time()
        streams = [torch.cuda.Stream() for _ in range(nst)]
        per_round = []
        detail = None
        for rnd in range(rounds):
            e0 = ix.error_count()
            outs = [(torch.empty((256, k), device="cuda"), torch.empty((256, k), dtype=torch.int64, device="cuda"))
                    for _ in range(nb)]
            ix.inflight = nst > 1 and os.environ.get("RACE_INFLIGHT", "1") != "0"
            try:
                torch.cuda.synchronize()
                if hog:
                    with torch.cuda.stream(side):
                        for _ in range(40):
                            hog_b.copy_(hog_a)
                for b in range(nb):
                    st = streams[b % nst]
                    if mix and b == 5:
                        with torch.cuda.stream(st):
                            Dq, Iq = ix.coarse_device(xd[b], stream=st.cuda_stream)
                            ix.search_preassigned_device(xd[b], k, Iq, Dq, stream=st.cuda_stream)
                    if coarse_only:
                        with torch.cuda.stream(st):
                            cq = ix.coarse_device(xd[b], stream=st.cuda_stream)
                        outs[b] = (cq[0], cq[1])
                    elif pre_only:
                        with torch.cuda.stream(st):
                            ix.search_preassigned_device(xd[b], k, cref[b][1], cref[b][0], outs[b][0], outs[b][1],
                                                         stream=st.cuda_stream)
                    else:
                        ix.search_device(xd[b], k, outs[b][0], outs[b][1], stream=st.cuda_stream)
                torch.cuda.synchronize()
            finally:
                ix.inflight = False
            bad_b, bad_rows, sent, nonfin = 0, 0, 0, 0
            for b in range(nb):
                D = outs[b][0].cpu().numpy()
                I = outs[b][1].cpu().numpy()
                Dr, Ir = refs[k][b]
                if coarse_only:
                    Dr, Ir = cref[b][0].cpu().numpy(), cref[b][1].cpu().numpy()
                rows = np.nonzero((I != Ir).any(axis=1) | (D != Dr).any(axis=1))[0]
                if len(rows):
                    bad_b += 1
                    bad_rows += len(rows)
                    sent += int((I[rows] == big).sum())
                    nonfin += int((~np.isfinite(D[rows])).sum())
                    if detail is None:
                        r = int(rows[0])
                        diff = np.nonzero((I[r] != Ir[r]) | (D[r] != Dr[r]))[0]
                        detail = {"round": rnd, "batch": b, "stream": b % nst, "row": r, "rows": rows[:8].tolist(),
                                  "first_diff_rank": int(diff[0]), "n_diff": int(len(diff)),
                                  "I": I[r, diff[:6]].tolist(), "I_ref": Ir[r, diff[:6]].tolist(),
                                  "D": D[r, diff[:6]].tolist(), "D_ref": Dr[r, diff[:6]].tolist()}
            per_round.append({"bad_batches": bad_b, "bad_rows": bad_rows, "sentinels": sent, "nonfinite": nonfin,
                              "err": ix.error_count() - e0})
        st, rp = ix.repair_stats()
        dbg = None
        lib = _lib.load()
        if hasattr(lib, "ivfpq_dbg_read"):  # debug variant (profiles/race_variants.py dbg)
            import ctypes
            buf = (ctypes.c_uint32 * (1 + 64 * 48))()
            lib.ivfpq_dbg_read(buf, 1)
            n = min(buf[0], 64)
            dbg = {"count": buf[0], "events": [list(buf[1 + 48 * e:1 + 48 * e + 31]) for e in range(min(n, 12))]}
        print(json.dumps({"k": k, "streams": nst, "hog": hog, "mix": mix, "rounds": rounds,
                          "mode": "coarse" if coarse_only else "preassigned" if pre_only else "search",
                          "inflight": nst > 1 and os.environ.get("RACE_INFLIGHT", "1") != "0",
                          "stale_reads_total": st, "repairs_total": rp, "log": ix.repair_log(64), "dbg": dbg,
                          "bad_batches": sum(r["bad_batches"] for r in per_round),
                          "bad_rounds": [dict(r, round=i) for i, r in enumerate(per_round) if r["bad_batches"] or r["err"]], "first": detail,
                          "s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
