#!/usr/bin/env python3
"""C5: per-stage latency of one RAG retrieval request
served by the MI355X engine behind the RALM wire format.

The reference times its RAG pipeline per stage (reranker_hf/advanced_rag.py:
230-276: retrieval, rerank, prompt build, llm; and RALM's "Retrieval" line,
ralm/retriever/serialization_utils.py commented timings).  Only the retrieval
stage is this build's path; rerank and LLM are out of scope.
For one request of B queries the retrieval stage splits into:

  client encode_request -> [server: decode, H2D, coarse, LUT+scan+top-k, D2H,
  encode_answer] -> client decode_answer

measured two ways:
  native  -- RetrievalService.handle -> ivfpq_serve_request (one C call: the
             request bytes go straight to HBM, the answer straight into the
             reply buffer); device stages from HIP events in the same call;
  python  -- the reference FaissServer's loop body restated over this engine:
             wire.decode_request + IndexIVFPQ.search + wire.encode_answer.

Shapes: the FaissServer docstring's RALM setting (faiss_server.py:5-9: d=512,
IVF32768,PQ32, nprobe=32, batch 32, k=10; synthetic base of --nb vectors) and
the C2 SIFT1M index at batch 32 and 1024.  Prints one JSON line per shape.
Usage: python profiles/rag_stages.py [--reps 200] [--nb 1000000]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "chameleon-rag-acceleration_amd"))

import numpy as np  # noqa: E402


def med_ms(ts):
    return float(np.median(ts) * 1e3)


def run_shape(name, ix, xq_all, B, k, nprobe, reps):
    from faiss_amd import wire
    from faiss_amd.server import RetrievalService

    d = ix.d
    svc = RetrievalService(ix, batch_size=B, default_k=k, nprobe=nprobe)
    nb = xq_all.shape[0] // B
    reqs = [bytes(wire.encode_request(np.ascontiguousarray(xq_all[i * B:(i + 1) * B]), k, B, d)) for i in range(nb)]
    for i in range(5):
        svc.handle(reqs[i % nb])
    t_enc, t_srv, t_dec = [], [], []
    for r in range(reps):
        q = xq_all[(r % nb) * B:(r % nb + 1) * B]
        t0 = time.perf_counter()
        msg = wire.encode_request(q, k, B, d)
        t1 = time.perf_counter()
        ans = svc.handle(msg)
        t2 = time.perf_counter()
        wire.decode_answer(ans, k, B)
        t3 = time.perf_counter()
        t_enc.append(t1 - t0)
        t_srv.append(t2 - t1)
        t_dec.append(t3 - t2)
    # device stage split in a separate pass (each recorded event costs a few us)
    ix.set_timing(True)
    for r in range(reps):
        svc.handle(reqs[r % nb])
    ix.set_timing(False)
    st = ix.get_timing()
    dev = {s: (v[0] / max(v[1], 1)) for s, v in st.items() if v[1]}
    # python path (the reference server's loop body over this engine)
    t_pdec, t_psearch, t_penc = [], [], []
    for r in range(reps):
        m = reqs[r % nb]
        t0 = time.perf_counter()
        kk, q = wire.decode_request(m, B, d)
        t1 = time.perf_counter()
        D, I = ix.search(q, kk)
        t2 = time.perf_counter()
        wire.encode_answer(I, D, kk, B)
        t3 = time.perf_counter()
        t_pdec.append(t1 - t0)
        t_psearch.append(t2 - t1)
        t_penc.append(t3 - t2)
    srv = med_ms(t_srv)
    dev_sum = dev.get("coarse", 0) + dev.get("tables", 0) + dev.get("scan", 0)
    return {
        "shape": name, "batch": B, "k": k, "nprobe": nprobe, "d": d, "nlist": ix.nlist, "M": ix.M,
        "ntotal": int(ix.ntotal), "reps": reps,
        "native_ms": {"client_encode_request": med_ms(t_enc), "server_handle": srv,
                      "client_decode_answer": med_ms(t_dec),
                      "device_coarse": dev.get("coarse"), "device_tables": dev.get("tables"),
                      "device_scan_topk": dev.get("scan"),
                      "host_and_pcie (handle - device stages)": srv - dev_sum},
        "native_requests_per_s": 1e3 / srv, "native_queries_per_s": B * 1e3 / srv,
        "python_ms": {"decode_request": med_ms(t_pdec), "search": med_ms(t_psearch),
                      "encode_answer": med_ms(t_penc),
                      "total": med_ms(t_pdec) + med_ms(t_psearch) + med_ms(t_penc)},
        "note": "medians over reps, timed without events; device stages are HIP-event means from a separate pass; "
                "rerank / prompt / LLM stages of the RAG pipeline are out of scope",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--nb", type=int, default=1_000_000)
    ap.add_argument("--ralm-nt", type=int, default=200_000)
    ap.add_argument("--niter", type=int, default=6)
    ap.add_argument("--skip-ralm", action="store_true")
    a = ap.parse_args()
    import faiss_amd as faiss
    from faiss_amd import datasets

    out = []
    # C2 index (SIFT1M-shaped)
    xt = datasets.synthetic_sift_like(100_000, 128, seed=4321)
    xb = datasets.synthetic_sift_like(a.nb, 128, seed=1234)
    xq = datasets.synthetic_sift_like(10_240, 128, seed=123)
    ix = faiss.index_factory(128, "IVF1024,PQ16", device=0)
    ix.niter_coarse = ix.niter_pq = 25
    ix.train(xt)
    ix.add(xb)
    del xb
    ix.nprobe = 16
    for B in (32, 1024):
        r = run_shape("C2 SIFT1M-shaped IVF1024,PQ16", ix, xq, B, 10, 16, a.reps)
        print(json.dumps(r), flush=True)
        out.append(r)
    del ix
    if not a.skip_ralm:
        # RALM FaissServer setting (faiss_server.py:5-9): d=512, IVF32768,PQ32, nprobe 32, batch 32, k 10
        d = 512
        xt = datasets.synthetic_sift_like(a.ralm_nt, d, seed=11)
        ix = faiss.index_factory(d, "IVF32768,PQ32", device=0)
        ix.niter_coarse = ix.niter_pq = a.niter
        t0 = time.time()
        ix.train(xt)
        print(f"[rag] RALM-shaped train {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
        for i0 in range(0, a.nb, 250_000):
            ix.add(datasets.synthetic_sift_like(min(250_000, a.nb - i0), d, seed=100 + i0))
        ix.nprobe = 32
        xq = datasets.synthetic_sift_like(32 * 64, d, seed=7)
        r = run_shape("RALM FaissServer IVF32768,PQ32 d=512", ix, xq, 32, 10, 32, a.reps)
        print(json.dumps(r), flush=True)
        out.append(r)


if __name__ == "__main__":
    main()
