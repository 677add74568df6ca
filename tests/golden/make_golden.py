"""Generate the committed golden fixtures under tests/golden/ (run in the dev
container only: it reads /root/reference, which does not exist on the GPU box).

Two kinds of fixture are written:

1. ``ivfpq_<case>.npz`` — a small trained IVF-PQ index (centroids, PQ codebook,
   inverted lists), queries, and three result sets for the same queries:
   * ``nb_ids / nb_dists``: the reference's own NumPy IVF-PQ search
     (``Chameleon/Faiss_experiments/my_faiss_extract_scripts/IVFPQ_1B_search.ipynb``
     cell 20: ``search_batch_query`` :8019-8030 → ``search_single_query``
     :7986-8018 → ``construct_distance_table`` :7929-7946 /
     ``estimate_distances`` :7948-7985), executed here from the notebook file
     with a stub ``get_invlist`` over our inverted lists (the original reads
     Faiss invlists via ``faiss.rev_swig_ptr``);
   * ``or_D / or_I``: the C oracle (oracle/ivfpq_oracle.c) at generation time,
     so later runs can check the oracle build is unchanged bit for bit;
   * ``or_lists / or_dis0``: the oracle's coarse assignment.
2. ``lut_kat.npz`` — the FPGA LUT known-answer test data
   (``Chameleon/retrieval_accelerator/LUT_construction_PEs/
   LUT_construction_PE_D128_M32/src/host.cpp``: codebook ``i % 256`` :44-46,
   query :58-64, centroid :73-79, software LUT :88-109), parsed from that file.

The index itself is trained by the oracle's own k-means (Faiss training is not
reproducible without Faiss; SURVEY §7 "Hard parts").
"""
from __future__ import annotations

import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "chameleon-rag-acceleration_amd"))

from oracle import oracle as O  # noqa: E402
from faiss_amd import datasets  # noqa: E402

REF = "/root/reference/Chameleon"
NOTEBOOK = REF + "/Faiss_experiments/my_faiss_extract_scripts/IVFPQ_1B_search.ipynb"
KAT_HOST = REF + "/retrieval_accelerator/LUT_construction_PEs/LUT_construction_PE_D128_M32/src/host.cpp"

CASES = [
    # name, d, M, nlist, nb, nt, nq, nprobe, k, (n_centres, sigma) of the synthetic data
    ("d128_m16", 128, 16, 64, 20000, 8000, 24, 8, 10, (200, 16.0)),
    ("d64_m32_dsub2", 64, 32, 32, 8000, 4000, 16, 4, 20, (200, 16.0)),
    # spread-out data: with 200 tight clusters the 8-byte codes repeat and most
    # of the top-k are exact ties (round-1 review)
    ("d96_m8_dsub12", 96, 8, 32, 8000, 4000, 16, 6, 16, (4000, 32.0)),
]


def load_notebook_search():
    nb = json.load(open(NOTEBOOK))
    src = "".join(nb["cells"][20]["source"])
    assert "def search_batch_query" in src
    ns = {"np": np}
    exec(compile(src, "IVFPQ_1B_search.ipynb:cell20", "exec"), ns)
    return ns


def make_case(ns, name, d, M, nlist, nb, nt, nq, nprobe, k, gen):
    nc, sigma = gen
    xt = datasets.synthetic_sift_like(nt, d, seed=4321, n_centres=nc, sigma=sigma)
    xb = datasets.synthetic_sift_like(nb, d, seed=1234, n_centres=nc, sigma=sigma)
    xq = datasets.synthetic_sift_like(nq, d, seed=123, n_centres=nc, sigma=sigma)
    ix = O.OracleIVFPQ(d, nlist, M)
    ix.train(xt, niter_coarse=10, niter_pq=10, seed=1234)
    ids = (5 * np.arange(nb, dtype=np.int64) + 11)[::-1].copy()
    ix.add_with_ids(xb, ids)
    ix.nprobe = nprobe
    or_dis0, or_lists = O.coarse_search(xq, ix.centroids, nprobe)
    or_D, or_I = ix.search(xq, k)

    class _Inv:
        pass

    inv = _Inv()
    ns["invlists"] = inv
    ns["get_invlist"] = lambda _inv, l: (ix.list_ids[l], ix.list_codes[l])
    nb_ids = np.full((nq, k), -1, np.int64)
    nb_dists = np.full((nq, k), np.inf, np.float64)
    ids_b, dists_b = ns["search_batch_query"](xq, nprobe, k, ix.centroids, ix.codebook)
    for q in range(nq):
        nb_ids[q, :len(ids_b[q])] = ids_b[q]
        nb_dists[q, :len(dists_b[q])] = dists_b[q]
    off, codes, lids = ix.invlists_flat()
    path = os.path.join(HERE, f"ivfpq_{name}.npz")
    np.savez_compressed(
        path, d=d, M=M, nlist=nlist, nprobe=nprobe, k=k, centroids=ix.centroids, codebook=ix.codebook,
        list_off=off, codes=codes, ids=lids, xq=xq, or_D=or_D, or_I=or_I, or_lists=or_lists, or_dis0=or_dis0,
        nb_ids=nb_ids, nb_dists=nb_dists)
    agree = (nb_ids == or_I).mean()
    print(f"{name}: oracle-vs-notebook id agreement {agree:.4f}, "
          f"max rel dist diff {np.max(np.abs(nb_dists - or_D) / np.maximum(1, np.abs(nb_dists))):.2e} -> {path}")


def parse_c_array(src, name):
    m = re.search(r"float\s+" + name + r"\s*\[D\]\s*=\s*\{([^}]*)\}", src)
    return np.array([int(t) for t in m.group(1).replace("\n", " ").split(",") if t.strip()], np.float32)


def make_kat():
    src = open(KAT_HOST).read()
    q = parse_c_array(src, "query_vec_data")
    c = parse_c_array(src, "center_vec_data")
    assert q.shape == (128,) and c.shape == (128,)
    out = {"query": q, "center": c}
    D = 128
    for M in (32, 16):
        dsub = D // M
        # host.cpp:44-46: product_quantizer[i] = i % 256 in layout M x 256 x (D/M)
        cb = (np.arange(D * 256) % 256).astype(np.float32).reshape(M, 256, dsub)
        diff = (q - c).astype(np.float32)
        lut = np.zeros((256, M), np.float32)  # host.cpp:91-109, float accumulation in c order
        for j in range(256):
            for m in range(M):
                acc = np.float32(0)
                for t in range(dsub):
                    e = np.float32(diff[m * dsub + t] - cb[m, j, t])
                    acc = np.float32(acc + np.float32(e * e))
                lut[j, m] = acc
        out[f"codebook_M{M}"] = cb
        out[f"lut_M{M}"] = lut
    path = os.path.join(HERE, "lut_kat.npz")
    np.savez_compressed(path, **out)
    print("KAT ->", path)


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit("make_golden.py needs /root/reference (dev container only)")
    make_kat()
    ns = load_notebook_search()
    only = sys.argv[1:]  # optional case names to regenerate
    for case in CASES:
        if not only or case[0] in only:
            make_case(ns, *case)
