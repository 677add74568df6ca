#!/usr/bin/env python3
"""r05: autopsy of a wrong batch under batches-in-flight (race_diag's index, k = 10).

Each round issues one 256-query batch on each of `nst` streams with the handle's
inflight mode on, so every batch is the last one its workspace ran; a batch that
differs from its search alone is examined through ivfpq_debug_workspace: for every
true top-k label the result lost, the probe whose list holds it, the scan wave
that covered its position ((i mod 256) / 64), and that wave's partial list as the
merge read it (tag, entries, keys) -- whether the candidate was never admitted
(its key above what the list kept: a bound problem) or the list itself is wrong.
Prints one JSON line per examined row (at most AUT_MAX)."""
import ctypes
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "chameleon-rag-acceleration_amd"))

A = 0x9E3779B1
MASK = 0x0FFFFFFF


def main():
    import numpy as np
    import torch

    import faiss_amd as faiss
    from faiss_amd import _lib, datasets

    k = 10
    nst = int(os.environ.get("AUT_STREAMS", "3"))
    rounds = int(os.environ.get("AUT_ROUNDS", "3000"))
    amax = int(os.environ.get("AUT_MAX", "12"))
    lib = _lib.load()
    xt = datasets.synthetic_sift_like(20_000, 64, seed=4321, n_centres=20_000)
    xb = datasets.synthetic_sift_like(100_000, 64, seed=1234, n_centres=20_000)
    xq = datasets.synthetic_sift_like(24 * 256, 64, seed=123, n_centres=20_000)
    ix = faiss.index_factory(64, "IVF256,PQ8", device=0)
    ix.niter_coarse = ix.niter_pq = 8
    ix.train(xt)
    ix.add(xb)
    np_ = 12
    ix.nprobe = np_
    nb = 24
    xd = torch.from_numpy(xq).cuda().view(nb, 256, 64)
    sizes = ix.invlists.list_sizes()
    off = np.concatenate([[0], np.cumsum(sizes)])
    lab_list = np.empty(ix.ntotal, np.int64)
    lab_pos = np.empty(ix.ntotal, np.int64)
    for l in range(256):
        ids = np.sort(ix.invlists.get_ids(l))
        lab_list[ids] = l
        lab_pos[ids] = np.arange(len(ids))
    ref, cref = [], []
    for b in range(nb):
        D, I = ix.search_device(xd[b], k)
        Dq, Iq = ix.coarse_device(xd[b])
        torch.cuda.synchronize()
        ref.append((D.cpu().numpy(), I.cpu().numpy()))
        cref.append(Iq.cpu().numpy())
    streams = [torch.cuda.Stream() for _ in range(nst)]
    shandles = [s.cuda_stream for s in streams]

    def ws_buf(ws, what, dtype):
        nbytes = ctypes.c_int64(0)
        _lib.check(lib.ivfpq_debug_workspace(ix._h, ws, what, None, 0, ctypes.byref(nbytes)))
        a = np.empty(nbytes.value // np.dtype(dtype).itemsize, dtype)
        _lib.check(lib.ivfpq_debug_workspace(ix._h, ws, what, a.ctypes.data, a.nbytes, ctypes.byref(nbytes)))
        return a

    examined, bad_batches, batches = 0, 0, 0
    for rnd in range(rounds):
        bs = [(rnd * nst + j) % nb for j in range(nst)]
        outs = [(torch.empty((256, k), device="cuda"), torch.empty((256, k), dtype=torch.int64, device="cuda"))
                for _ in range(nst)]
        torch.cuda.synchronize()
        ix.inflight = True
        try:
            for j in range(nst):
                ix.search_device(xd[bs[j]], k, outs[j][0], outs[j][1], stream=shandles[j])
            torch.cuda.synchronize()
        finally:
            pass
        batches += nst
        for j in range(nst):
            b = bs[j]
            I = outs[j][1].cpu().numpy()
            D = outs[j][0].cpu().numpy()
            rows = np.nonzero((I != ref[b][1]).any(1) | (D != ref[b][0]).any(1))[0]
            if not len(rows):
                continue
            bad_batches += 1
            if examined >= amax:
                continue
            # the workspace this stream used (inflight off would quiesce: read with it on)
            ws = None
            for w in range(3):
                if int(ws_buf(w, 8, np.uint64)[0]) == shandles[j]:
                    ws = w
            rec = {"round": rnd, "batch": b, "stream": j, "ws": ws, "rows": rows[:4].tolist()}
            if ws is None:
                print(json.dumps(rec), flush=True)
                continue
            epoch = int(ws_buf(ws, 7, np.uint64)[0])
            part = ws_buf(ws, 0, np.uint32).reshape(-1, 4)
            pn = ws_buf(ws, 1, np.uint32).reshape(-1, 2)
            qm = ws_buf(ws, 2, np.uint64)
            tau = ws_buf(ws, 3, np.uint64)
            rec["epoch"] = epoch
            for r in rows[:2]:
                r = int(r)
                lost = [int(x) for x in ref[b][1][r] if x not in set(I[r].tolist())]
                kth = float(ref[b][0][r, k - 1])
                tv = int(tau[r])
                te = (~(tv >> 32)) & 0xFFFFFFFF
                to = (tv & 0xFFFFFFFF) ^ 0x80000000
                to = to - (1 << 32) if to >= (1 << 31) else to
                tkey = np.array([to if to >= 0 else to ^ 0x7FFFFFFF], np.int32).view(np.float32)[0]
                info = {"row": r, "kth_true": kth, "tau_epoch": int(te), "tau_key": float(tkey),
                        "tau_below_kth": bool(te == epoch and tkey < kth), "qmask": hex(int(qm[r])), "lost": []}
                for x in lost[:3]:
                    l, i = int(lab_list[x]), int(lab_pos[x])
                    ps = np.nonzero(cref[b][r] == l)[0]
                    p = int(ps[0]) if len(ps) else -1
                    wv = (i % 256) // 64
                    xkey = float(ref[b][0][r][list(ref[b][1][r]).index(x)])
                    e = {"label": x, "key": xkey, "list": l, "pos": i, "probe": p, "wave": wv}
                    if p >= 0:
                        slot = (r * np_ + p) * 4 + wv
                        expect = (epoch * A + slot) & MASK
                        ents = part[slot * k:(slot + 1) * k]
                        keys = ents[:, 0].view(np.float32)
                        tags = ents[:, 1]
                        poss = (ents[:, 3].astype(np.int64) << 32) | ents[:, 2]
                        e.update({"tags_fresh": int(((tags & MASK) == expect).sum()), "writer_xcd": sorted(set((tags >> 28).tolist())),
                                  "n_entries": int((poss != -1).sum() if poss.dtype == np.int64 else 0),
                                  "keys": [float(v) for v in keys], "has_it": bool((poss == off[l] + i).any()),
                                  "probe_bit": bool((int(qm[r]) >> p) & 1)})
                    info["lost"].append(e)
                rec.setdefault("detail", []).append(info)
            examined += 1
            print(json.dumps(rec), flush=True)
        ix.inflight = False
    print(json.dumps({"summary": True, "batches": batches, "bad_batches": bad_batches}), flush=True)


if __name__ == "__main__":
    main()
