"""faiss.contrib.ivf_tools.search_preassigned, as called by the RALM retrievers
(``Chameleon/llm_inference_gpu/ralm/retriever/faiss_retriever.py:265``,
``ralm/server/faiss_server.py:208, 233``).

As in upstream Faiss of that era, ``coarse_dis=None`` means zeros: with
precomputed tables this drops |q - c|^2 from every distance;
pass the coarse distances to rank across lists correctly (the reference's own
``replacement_search_preassigned``, faiss_retriever.py:178-225).
"""
import numpy as np


def search_preassigned(index_ivf, xq, k, list_nos, coarse_dis=None):
    n = xq.shape[0]
    list_nos = np.ascontiguousarray(list_nos, dtype=np.int64)
    if list_nos.shape != (n, index_ivf.nprobe):
        raise RuntimeError(f"list_nos must have shape {(n, index_ivf.nprobe)}, got {list_nos.shape}")
    if coarse_dis is None:
        coarse_dis = np.zeros(list_nos.shape, dtype=np.float32)
    elif np.asarray(coarse_dis).shape != list_nos.shape:
        raise RuntimeError("coarse_dis must have the shape of list_nos")
    return index_ivf.search_preassigned(xq, k, list_nos, coarse_dis)
