#!/usr/bin/env python3
"""Host enqueue cost of one device search.

Builds a C2-shaped index (IVF1024,PQ16, d 128; 200k base vectors -- the host
work per call does not depend on the list sizes), then times, for 1024-query
batches at k = 10, nprobe 16:
  * py:      bench.py's step (faiss_amd search_device, Python validation + ctypes);
  * py+tm:   the same with bench.py's per-step set_timing call;
  * ctypes:  ivfpq_search_device called directly through ctypes (no Python checks);
each as (host seconds per call with no synchronization inside the loop, GPU
seconds per call from the synchronized total).  If host >= GPU per call, the
GPU waits for the host between launches.  One JSON line."""
import ctypes
import json
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "chameleon-rag-acceleration_amd"))


def main():
    import torch

    import faiss_amd as faiss
    from faiss_amd import _lib, datasets

    n_calls = int(os.environ.get("ENQ_CALLS", "400"))
    xt = datasets.synthetic_sift_like(50_000, 128, seed=4321, n_centres=200_000)
    xb = datasets.synthetic_sift_like(200_000, 128, seed=1234, n_centres=200_000)
    xq = datasets.synthetic_sift_like(4 * 1024, 128, seed=123, n_centres=200_000)
    ix = faiss.index_factory(128, "IVF1024,PQ16", device=0)
    ix.niter_coarse = ix.niter_pq = 8
    ix.train(xt)
    ix.add(xb)
    ix.nprobe = 16
    xd = torch.from_numpy(xq).cuda().view(4, 1024, 128)
    D = torch.empty((1024, 10), device="cuda")
    I = torch.empty((1024, 10), dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    lib = _lib.load()
    out = {}

    def run(name, fn):
        for i in range(20):
            fn(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n_calls):
            fn(i)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out[name] = {"host_us_per_call": (t1 - t0) * 1e6 / n_calls, "gpu_us_per_call": (t2 - t0) * 1e6 / n_calls}

    run("py", lambda i: ix.search_device(xd[i % 4], 10, D, I, stream=st.cuda_stream))

    def py_tm(i):
        ix.set_timing(i % 5 == 0, lists_only=True)
        ix.search_device(xd[i % 4], 10, D, I, stream=st.cuda_stream)

    run("py+tm", py_tm)
    ix.set_timing(False)
    ix.get_timing()
    ptrs = [xd[b].data_ptr() for b in range(4)]
    h = ix._h
    s = ctypes.c_void_p(st.cuda_stream)
    dp, ip_ = D.data_ptr(), I.data_ptr()
    run("ctypes", lambda i: lib.ivfpq_search_device(h, 1024, ptrs[i % 4], 10, dp, ip_, s))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
