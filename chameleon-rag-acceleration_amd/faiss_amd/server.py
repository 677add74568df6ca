"""Request handling of Chameleon's ``FaissServer`` on the MI355X engine.

``Chameleon/llm_inference_gpu/ralm/server/faiss_server.py`` receives fixed-size
requests over TCP, decodes them (``serialization_utils``), runs
``index.search`` (``retrieve``, :170-218) or ``search_preassigned`` with the
client's coarse lists (``retrieve_with_lists``, :220-239) and sends the encoded
answer back (``start``, :241-277).  ``RetrievalService`` is that middle part:
``handle(request_bytes) -> answer_bytes``, computed by one native call
(``IndexIVFPQ.serve_request`` -> ``ivfpq_serve_request``).  The socket loop
itself (accept, ``recv`` until ``query_msg_len`` bytes, ``send``) is the
caller's and is out of scope here; it needs only
``query_msg_len`` and ``handle``.

``retrieve`` / ``retrieve_with_lists`` keep FaissServer's signatures and return
its ``{"id": I, "dist": D}`` dicts.
"""
from __future__ import annotations

import time
from typing import Optional

import numpy as np

from . import wire


class RetrievalService:
    def __init__(self, index, batch_size: int = 1, dim: Optional[int] = None, default_k: int = 10,
                 nprobe: int = 1, request_with_lists: int = 0):
        self.index = index
        self.batch_size = int(batch_size)
        self.dim = int(index.d if dim is None else dim)
        if self.dim != index.d:
            raise RuntimeError(f"dim={self.dim} does not match the index (d={index.d})")  # faiss_server.py:64
        self.default_k = int(default_k)
        self.request_with_lists = int(request_with_lists)
        self.set_nprobe(nprobe)
        if self.request_with_lists:
            self.query_msg_len = wire.request_message_length_with_lists(self.batch_size, self.dim, self.nprobe)
        else:
            self.query_msg_len = wire.request_message_length(self.batch_size, self.dim)
        self.answer_msg_len = wire.answer_message_len(self.default_k, self.batch_size)
        self._answer = bytearray(self.answer_msg_len)
        self.served = 0
        self.busy_s = 0.0

    def set_nprobe(self, nprobe: int):
        self.nprobe = int(nprobe)
        self.index.nprobe = self.nprobe

    # FaissServer.retrieve / retrieve_with_lists (host numpy in and out)
    def retrieve(self, query: np.ndarray, nprobe: Optional[int] = None, k: Optional[int] = None):
        k = self.default_k if k is None else k
        if nprobe is not None:
            self.set_nprobe(nprobe)
        if query.shape[1] != self.dim:
            raise RuntimeError(f"query dim {query.shape[1]} != {self.dim}")
        D, I = self.index.search(query, k)
        return {"id": I, "dist": D}

    def retrieve_with_lists(self, query: np.ndarray, list_IDs: np.ndarray, k: Optional[int] = None):
        k = self.default_k if k is None else k
        if query.shape[1] != self.dim or list_IDs.shape[0] != query.shape[0]:
            raise RuntimeError("query / list_IDs shape mismatch")
        if list_IDs.dtype != np.int64:
            raise RuntimeError("list_IDs must be int64")  # faiss_server.py:231
        D, I = self.index.search_preassigned(query, k, list_IDs)
        return {"id": I, "dist": D}

    def handle(self, request) -> bytearray:
        """One request message -> its answer message (FaissServer.start's loop body).
        The answer buffer is reused across calls: send or copy it before the next call."""
        if len(request) != self.query_msg_len:
            raise RuntimeError(f"request is {len(request)} bytes, expected {self.query_msg_len}")
        k = wire.peek_k(request, self.request_with_lists)
        if k != self.default_k:  # faiss_server.py:260, :266 assert k == default_k
            raise RuntimeError(f"request asks for k={k}, the server serves k={self.default_k}")
        t0 = time.perf_counter()
        out = self.index.serve_request(request, self.batch_size, self.dim, with_lists=bool(self.request_with_lists),
                                       nprobe=self.nprobe, out=self._answer)
        self.busy_s += time.perf_counter() - t0
        self.served += 1
        return out
