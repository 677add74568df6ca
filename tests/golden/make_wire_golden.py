"""Generate tests/golden/wire_messages.npz: RALM wire-format messages produced by
the reference's own encoder (run in the dev container only; it imports
``Chameleon/llm_inference_gpu/ralm/retriever/serialization_utils.py`` from
/root/reference, which does not exist on the GPU box).

Stored (data only, no reference source): the inputs (queries, list ids, k,
answer ids/distances) and the exact bytes of ``encode_request``,
``encode_request_with_lists`` and ``encode_answer`` for two shapes: the
reference test's own shape (``tests/test_retriever.py:15-40``: batch 32, dim
512, k 2, nprobe 10) and an odd one (batch 3, dim 5, nprobe 3, k 7: list ids
at a byte offset that is not 8-aligned).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/Chameleon/llm_inference_gpu"


def main():
    sys.path.insert(0, REF)
    from ralm.retriever import serialization_utils as S  # noqa: E402

    rng = np.random.default_rng(2024)
    out = {}
    for tag, (b, dim, k, np_) in {"t": (32, 512, 2, 10), "odd": (3, 5, 7, 3)}.items():
        q = rng.random((b, dim), dtype=np.float32)
        lists = rng.integers(0, 100, size=(b, np_), dtype=np.int64)
        ids = np.arange(b * k, dtype=np.int64).reshape(b, k) * 7 - 3
        dis = rng.standard_normal((b, k), dtype=np.float32)
        out[f"{tag}_shape"] = np.array([b, dim, k, np_], np.int64)
        out[f"{tag}_queries"] = q
        out[f"{tag}_lists"] = lists
        out[f"{tag}_ids"] = ids
        out[f"{tag}_dis"] = dis
        out[f"{tag}_req"] = np.frombuffer(bytes(S.encode_request(q, k, b, dim)), np.uint8)
        out[f"{tag}_req_lists"] = np.frombuffer(bytes(S.encode_request_with_lists(q, lists, b, dim, np_, k)),
                                                np.uint8)
        out[f"{tag}_answer"] = np.frombuffer(bytes(S.encode_answer(ids, dis, k, b)), np.uint8)
        out[f"{tag}_lens"] = np.array([S.request_message_length(b, dim),
                                       S.request_message_length_with_lists(b, dim, np_),
                                       S.answer_message_len(k, b)], np.int64)
    np.savez_compressed(os.path.join(HERE, "wire_messages.npz"), **out)
    print("wrote", os.path.join(HERE, "wire_messages.npz"))


if __name__ == "__main__":
    main()
