"""RALM retrieval wire format (drop-in for ``ralm.retriever.serialization_utils``).

Chameleon's GPU LLM workers talk to ``FaissServer`` over TCP with fixed-size
binary messages (``Chameleon/llm_inference_gpu/ralm/retriever/serialization_utils.py``).
This module produces and parses the same bytes, so a client or server keeps its
code and swaps the import.  Layouts (header integers big-endian int32, arrays
in the host's native order, as ``ndarray.tobytes`` writes them):

=====================  ===============================================================
request                ``k`` | queries f32 [batch][dim]                     (:17-18, :38-67)
request with lists     ``batch, dim, nprobe, k`` | queries | lists i64 [batch][nprobe]
                                                                            (:20-22, :69-94)
answer                 ids i64 [batch][k] | distances f32 [batch][k]         (:34-35, :223-290)
=====================  ===============================================================

The server side of the GPU path does not go through these Python helpers:
``IndexIVFPQ.serve_request`` hands the raw request to the native library
(``ivfpq_serve_request``), which copies the query bytes straight to HBM and the
results straight from HBM into the answer message.
"""
from __future__ import annotations

import struct
from typing import Tuple

import numpy as np

BYTE_ORDER_PY = "big"  # header integers (serialization_utils.py:5)
BYTE_ORDER_NP = "C"  # array order of tobytes (:6)

N_BYTES_K = 4
N_BYTES_PER_QUERY = 4  # per query element (float32)
N_BYTES_PER_IDX = 8
N_BYTES_PER_DIST = 4
N_BYTES_INT32 = 4
N_BYTES_FLOAT32 = 4
N_BYTES_AXI = 64

_HDR1 = struct.Struct(">i")  # k
_HDR4 = struct.Struct(">iiii")  # batch, dim, nprobe, k


def request_message_length(batch_size: int, dim: int) -> int:
    return N_BYTES_K + batch_size * dim * N_BYTES_PER_QUERY


def request_message_length_with_lists(batch_size: int, dim: int, nprobe: int) -> int:
    return _HDR4.size + batch_size * (dim * N_BYTES_FLOAT32 + nprobe * N_BYTES_PER_IDX)


def answer_message_len(k: int, batch_size: int) -> int:
    return batch_size * k * (N_BYTES_PER_IDX + N_BYTES_PER_DIST)


def encode_request(batch_of_queries: np.ndarray, k: int, batch_size: int, dim: int) -> bytearray:
    """k + queries (the plain request; FaissServer then runs ``index.search``)."""
    assert batch_of_queries.shape == (batch_size, dim)
    q = np.ascontiguousarray(batch_of_queries)
    out = bytearray(request_message_length(batch_size, dim))
    _HDR1.pack_into(out, 0, int(k))
    out[N_BYTES_K:] = q.tobytes(order=BYTE_ORDER_NP)
    return out


def encode_request_with_lists(batch_of_queries: np.ndarray, list_IDs: np.ndarray, batch_size: int, dim: int,
                              nprobe: int, k: int) -> bytearray:
    """Header (batch, dim, nprobe, k) + queries + the coarse lists to scan (FaissServer
    runs ``search_preassigned``)."""
    assert batch_of_queries.shape == (batch_size, dim)
    assert list_IDs.shape == (batch_size, nprobe)
    assert batch_of_queries.dtype == np.float32
    lists = np.ascontiguousarray(list_IDs, dtype=np.int64)
    out = bytearray(request_message_length_with_lists(batch_size, dim, nprobe))
    _HDR4.pack_into(out, 0, int(batch_size), int(dim), int(nprobe), int(k))
    q0 = _HDR4.size
    q1 = q0 + batch_size * dim * N_BYTES_FLOAT32
    out[q0:q1] = np.ascontiguousarray(batch_of_queries).tobytes(order=BYTE_ORDER_NP)
    out[q1:q1 + batch_size * nprobe * N_BYTES_PER_IDX] = lists.tobytes(order=BYTE_ORDER_NP)
    return out


def decode_request(serialized_request, batch_size: int, dim: int) -> Tuple[int, np.ndarray]:
    """-> (k, queries f32 [batch_size][dim]) (a view of the message bytes)."""
    (k,) = _HDR1.unpack_from(serialized_request, 0)
    q = np.frombuffer(serialized_request, dtype=np.float32, offset=N_BYTES_K, count=batch_size * dim)
    return int(k), q.reshape(batch_size, dim)


def decode_request_with_lists(serialized_request, batch_size: int, dim: int,
                              nprobe: int) -> Tuple[int, np.ndarray, np.ndarray]:
    """-> (k, queries f32 [batch][dim], list ids i64 [batch][nprobe]); the header's
    shape must equal the server's (batch_size, dim, nprobe)."""
    b, d, p, k = _HDR4.unpack_from(serialized_request, 0)
    assert b == batch_size
    assert d == dim
    assert p == nprobe
    q0 = _HDR4.size
    q = np.frombuffer(serialized_request, dtype=np.float32, offset=q0, count=batch_size * dim)
    # the ids start at 16 + 4*batch*dim bytes: not 8-byte aligned for odd batch*dim, so copy
    raw = bytes(memoryview(serialized_request)[q0 + batch_size * dim * N_BYTES_FLOAT32:
                                               q0 + batch_size * dim * N_BYTES_FLOAT32 +
                                               batch_size * nprobe * N_BYTES_PER_IDX])
    lists = np.frombuffer(raw, dtype=np.int64).reshape(batch_size, nprobe)
    return int(k), q.reshape(batch_size, dim), lists


def encode_answer(indices: np.ndarray, distances: np.ndarray, k: int, batch_size: int) -> bytearray:
    """ids (int64) then distances (float32), each [batch_size][k]."""
    assert indices.shape == (batch_size, k)
    assert indices.dtype == np.int64
    assert distances.shape == (batch_size, k)
    assert distances.dtype == np.float32
    out = bytearray(answer_message_len(k, batch_size))
    split = batch_size * k * N_BYTES_PER_IDX
    out[:split] = np.ascontiguousarray(indices).tobytes()
    out[split:] = np.ascontiguousarray(distances).tobytes()
    return out


def decode_answer(serialized_answer, k: int, batch_size: int) -> Tuple[np.ndarray, np.ndarray]:
    """-> (indices i64 [batch_size][k], distances f32 [batch_size][k])."""
    split = batch_size * k * N_BYTES_PER_IDX
    ids = np.frombuffer(serialized_answer, dtype=np.int64, count=batch_size * k)
    dis = np.frombuffer(serialized_answer, dtype=np.float32, offset=split, count=batch_size * k)
    return ids.reshape(batch_size, k), dis.reshape(batch_size, k)


def peek_k(serialized_request, with_lists: bool) -> int:
    """k of a request without decoding the arrays."""
    if with_lists:
        return int(_HDR4.unpack_from(serialized_request, 0)[3])
    return int(_HDR1.unpack_from(serialized_request, 0)[0])
