"""CPU sweep of the synthetic generator's (n_centres, sigma) for IVF1024,PQ16
recall vs nprobe (numpy k-means training + the oracle's encode/search)."""
import sys, time, json
import numpy as np
R = __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, R + "/chameleon-rag-acceleration_amd")
from faiss_amd import datasets
from oracle import oracle as O

def kmeans(x, k, niter, seed):
    rng = np.random.default_rng(seed)
    c = x[rng.choice(x.shape[0], k, replace=False)].copy()
    xn = (x * x).sum(1)
    for it in range(niter):
        cn = (c * c).sum(1)
        a = np.empty(x.shape[0], np.int64)
        for i0 in range(0, x.shape[0], 20000):
            d = xn[i0:i0+20000, None] + cn[None] - 2 * x[i0:i0+20000] @ c.T
            a[i0:i0+20000] = d.argmin(1)
        cnt = np.bincount(a, minlength=k)
        s = np.zeros_like(c)
        np.add.at(s, a, x)
        nz = cnt > 0
        c[nz] = s[nz] / cnt[nz, None]
    return c.astype(np.float32)

def run(nc, sigma, nb=1_000_000, nq=2000):
    t0 = time.time()
    g = lambda n, seed: datasets.synthetic_sift_like(n, 128, seed=seed, n_centres=nc, sigma=sigma)
    xt, xb, xq = g(100_000, 4321), g(nb, 1234), g(nq, 123)
    cent = kmeans(xt, 1024, 10, 0)
    ox = O.OracleIVFPQ(128, 1024, 16)
    # residuals of xt
    cn = (cent * cent).sum(1)
    a = (((xt * xt).sum(1)[:, None] + cn[None] - 2 * xt @ cent.T)).argmin(1)
    r = xt - cent[a]
    cb = np.stack([kmeans(np.ascontiguousarray(r[:, 8*m:8*m+8]), 256, 10, m + 1) for m in range(16)])
    ox.set_trained(cent, cb)
    lo, co = ox.encode(xb)
    ox.add_preencoded(lo, co, np.arange(nb, dtype=np.int64))
    xb64 = xb.astype(np.float32)
    bn = (xb64 * xb64).sum(1)
    gt = np.empty(nq, np.int64)
    for i0 in range(0, nq, 500):
        d = bn[None] - 2 * xq[i0:i0+500] @ xb64.T
        gt[i0:i0+500] = d.argmin(1)
    out = {"n_centres": nc, "sigma": sigma}
    for p in (1, 2, 4, 8, 16, 32):
        ox.nprobe = p
        D, I = ox.search(xq, 10)
        out[f"np{p}"] = (round(float((I[:, 0] == gt).mean()), 4), round(float((I == gt[:, None]).any(1).mean()), 4))
    out["s"] = round(time.time() - t0, 1)
    print(json.dumps(out), flush=True)

for spec in sys.argv[1:]:
    nc, sg = spec.split(":")
    run(int(nc), float(sg))
