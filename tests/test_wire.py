"""RALM wire format: faiss_amd.wire against messages the
reference's own encoder produced (tests/golden/make_wire_golden.py, from
ralm/retriever/serialization_utils.py), plus the round trips of the reference's
test (Chameleon/llm_inference_gpu/tests/test_retriever.py:15-52).  CPU only."""
import os

import numpy as np
import pytest

from faiss_amd import wire

SHAPES = ("t", "odd")


@pytest.fixture(scope="module")
def z(golden_dir):
    return dict(np.load(os.path.join(golden_dir, "wire_messages.npz")))


@pytest.mark.parametrize("tag", SHAPES)
def test_encoders_are_byte_identical_to_the_reference(z, tag):
    b, dim, k, np_ = (int(v) for v in z[f"{tag}_shape"])
    q, lists = z[f"{tag}_queries"], z[f"{tag}_lists"]
    assert bytes(wire.encode_request(q, k, b, dim)) == z[f"{tag}_req"].tobytes()
    assert bytes(wire.encode_request_with_lists(q, lists, b, dim, np_, k)) == z[f"{tag}_req_lists"].tobytes()
    assert bytes(wire.encode_answer(z[f"{tag}_ids"], z[f"{tag}_dis"], k, b)) == z[f"{tag}_answer"].tobytes()
    assert [wire.request_message_length(b, dim), wire.request_message_length_with_lists(b, dim, np_),
            wire.answer_message_len(k, b)] == list(z[f"{tag}_lens"])


@pytest.mark.parametrize("tag", SHAPES)
def test_decoders_read_reference_messages(z, tag):
    b, dim, k, np_ = (int(v) for v in z[f"{tag}_shape"])
    k1, q1 = wire.decode_request(z[f"{tag}_req"].tobytes(), b, dim)
    assert k1 == k and np.array_equal(q1, z[f"{tag}_queries"])
    k2, q2, l2 = wire.decode_request_with_lists(bytearray(z[f"{tag}_req_lists"].tobytes()), b, dim, np_)
    assert k2 == k and np.array_equal(q2, z[f"{tag}_queries"]) and np.array_equal(l2, z[f"{tag}_lists"])
    assert l2.dtype == np.int64 and q2.dtype == np.float32
    ids, dis = wire.decode_answer(z[f"{tag}_answer"].tobytes(), k, b)
    assert np.array_equal(ids, z[f"{tag}_ids"]) and np.array_equal(dis, z[f"{tag}_dis"])
    assert wire.peek_k(z[f"{tag}_req"].tobytes(), False) == k
    assert wire.peek_k(z[f"{tag}_req_lists"].tobytes(), True) == k


def test_round_trip_as_in_reference_test():
    # test_retriever.py:15-52 (batch 32, dim 512, k 2, nprobe 10)
    b, dim, k, np_ = 32, 512, 2, 10
    rng = np.random.default_rng(0)
    q = rng.random((b, dim), dtype=np.float32)
    lists = rng.integers(0, 100, size=(b, np_), dtype=np.int64)
    k1, q1 = wire.decode_request(wire.encode_request(q, k, b, dim), b, dim)
    k2, q2, l2 = wire.decode_request_with_lists(wire.encode_request_with_lists(q, lists, b, dim, np_, k), b, dim, np_)
    ids = np.arange(b * k, dtype=np.int64).reshape(b, k)
    dis = rng.standard_normal((b, k), dtype=np.float32)
    i3, d3 = wire.decode_answer(wire.encode_answer(ids, dis, k, b), k, b)
    assert k1 == k2 == k
    assert np.array_equal(q, q1) and np.array_equal(q, q2) and np.array_equal(lists, l2)
    assert np.array_equal(ids, i3) and np.array_equal(dis, d3)


def test_int32_lists_are_widened_and_errors_raise():
    b, dim, np_ = 2, 4, 3
    q = np.zeros((b, dim), np.float32)
    l32 = np.arange(b * np_, dtype=np.int32).reshape(b, np_)
    _, _, l = wire.decode_request_with_lists(wire.encode_request_with_lists(q, l32, b, dim, np_, 5), b, dim, np_)
    assert l.dtype == np.int64 and np.array_equal(l, l32)
    msg = wire.encode_request_with_lists(q, l32, b, dim, np_, 5)
    with pytest.raises(AssertionError):  # header shape != server shape
        wire.decode_request_with_lists(msg, b, dim, np_ + 1)
    with pytest.raises(AssertionError):
        wire.encode_request(q, 5, b + 1, dim)
    with pytest.raises(AssertionError):
        wire.encode_answer(np.zeros((b, 5), np.int32), np.zeros((b, 5), np.float32), 5, b)
