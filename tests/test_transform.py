"""OPQ / LinearTransform / IndexPreTransform on the CPU side (faiss_amd/transform.py).

* the oracle's t-ordered fmaf transform (or_linear_transform) against exact
  integer arithmetic, and against float64;
* OPQMatrix.train (host numpy, Faiss OPQMatrix::train's algorithm): orthonormal
  rows and a lower PQ reconstruction error than the identity start;
* the "IxPT" / "LTra" byte layout against a field-by-field assembly of upstream
  Faiss 1.7.1's writer order (index_write.cpp: write_index_header,
  write_VectorTransform, write_LinearTransform) -- parity unpinned: no
  Faiss-written OPQ file exists in the reference or this image;
* the factory keys the reference uses ("OPQ16,IVF262144,PQ16", bench_gpu_1bn.py:10).
"""
import struct

import numpy as np
import pytest

import faiss_amd as faiss
from faiss_amd import faiss_io
from faiss_amd.transform import OPQMatrix
from oracle import oracle as O


def test_oracle_linear_transform_exact_on_integers():
    rng = np.random.default_rng(0)
    x = rng.integers(-8, 9, (37, 24)).astype(np.float32)
    A = rng.integers(-8, 9, (16, 24)).astype(np.float32)
    b = rng.integers(-8, 9, 16).astype(np.float32)
    np.testing.assert_array_equal(O.linear_transform(x, A), (x.astype(np.int64) @ A.T.astype(np.int64)))
    np.testing.assert_array_equal(O.linear_transform(x, A, b),
                                  x.astype(np.int64) @ A.T.astype(np.int64) + b.astype(np.int64))


def test_oracle_linear_transform_float():
    rng = np.random.default_rng(1)
    x = rng.standard_normal((50, 128)).astype(np.float32)
    A = rng.standard_normal((64, 128)).astype(np.float32)
    np.testing.assert_allclose(O.linear_transform(x, A), x.astype(np.float64) @ A.T.astype(np.float64),
                               rtol=1e-4, atol=1e-4)


def _pq_mse(x, M, niter=10, seed=5):
    rng = np.random.default_rng(seed)
    cb = OPQMatrix._pq_kmeans(x.astype(np.float64), M, [None] * M, niter, rng)
    r = OPQMatrix._pq_recons(x.astype(np.float64), M, cb)
    return float(((x - r) ** 2).sum(1).mean())


def test_opq_train_rotation_is_orthonormal_and_helps():
    rng = np.random.default_rng(2)
    d, M, n = 32, 4, 4096
    # strongly correlated dims: PQ on the raw axes wastes its sub-spaces
    z = rng.standard_normal((n, 8)).astype(np.float32) * np.linspace(8, 1, 8, dtype=np.float32)
    x = (z @ rng.standard_normal((8, d)).astype(np.float32)
         + 0.05 * rng.standard_normal((n, d)).astype(np.float32)).astype(np.float32)
    opq = OPQMatrix(d, M)
    opq.niter, opq.niter_pq_0, opq.niter_pq = 6, 8, 2
    opq.train(x)
    A = opq.A.astype(np.float64)
    assert A.shape == (d, d) and opq.is_trained
    np.testing.assert_allclose(A @ A.T, np.eye(d), atol=1e-5)
    xc = x - x.mean(0)
    rotated = (xc.astype(np.float64) @ A.T).astype(np.float32)
    assert _pq_mse(rotated, M) < 0.9 * _pq_mse(xc, M)


def test_opq_reduced_output_dimension():
    rng = np.random.default_rng(3)
    x = rng.standard_normal((1000, 48)).astype(np.float32)
    opq = OPQMatrix(48, 4, 32)
    opq.niter, opq.niter_pq_0, opq.niter_pq = 2, 3, 1
    opq.train(x)
    assert opq.A.shape == (32, 48)
    np.testing.assert_allclose(opq.A.astype(np.float64) @ opq.A.T, np.eye(32), atol=1e-5)
    with pytest.raises(RuntimeError):
        OPQMatrix(32, 4, 48)
    with pytest.raises(RuntimeError):
        OPQMatrix(30, 4)


def test_factory_keys():
    pf = faiss.index.parse_factory
    assert pf("OPQ16,IVF262144,PQ16") == (262144, 16, 8, 16, -1)
    assert pf("OPQ16_64,IVF4096,PQ16") == (4096, 16, 8, 16, 64)
    assert pf("IVF1024,PQ16") == (1024, 16, 8)
    for bad in ("PCAR16,IVF1024,PQ16", "OPQ,IVF1024,PQ16", "OPQ16IVF1024,PQ16"):
        with pytest.raises(RuntimeError):
            pf(bad)


def _ltra(A, b, d_in, d_out):
    A = np.zeros(0, np.float32) if A is None else A.reshape(-1)
    bb = np.zeros(0, np.float32) if b is None else b
    return (b"LTra" + struct.pack("<B", int(b is not None)) + struct.pack("<Q", A.size) + A.tobytes()
            + struct.pack("<Q", bb.size) + bb.tobytes() + struct.pack("<i", d_in) + struct.pack("<i", d_out)
            + struct.pack("<B", 1))


def _tiny_ivfpq(d, seed=0):
    rng = np.random.default_rng(seed)
    nlist, M = 2, 2
    cent = rng.standard_normal((nlist, d)).astype(np.float32)
    cb = rng.standard_normal((M, 256, d // M)).astype(np.float32)
    lists = [(np.array([5, 9], np.int64), rng.integers(0, 256, (2, M)).astype(np.uint8)),
             (np.array([1], np.int64), rng.integers(0, 256, (1, M)).astype(np.uint8))]
    return faiss_io.serialize_ivfpq(d, nlist, 2, M, 8, 1, cent, cb, lists), lists


@pytest.mark.parametrize("bias", [False, True])
def test_pretransform_layout_matches_faiss_writer_order(bias):
    rng = np.random.default_rng(4)
    d_in, d_out = 12, 8
    A = rng.standard_normal((d_out, d_in)).astype(np.float32)
    b = rng.standard_normal(d_out).astype(np.float32) if bias else None
    sub, lists = _tiny_ivfpq(d_out)
    got = faiss_io.serialize_pretransform(d_in, 1, [(A, b, d_in, d_out, True)], sub, 3)
    hdr = struct.pack("<i", d_in) + struct.pack("<q", 3) + struct.pack("<qq", 1 << 20, 1 << 20) \
        + struct.pack("<B", 1) + struct.pack("<i", 1)
    want = b"IxPT" + hdr + struct.pack("<i", 1) + _ltra(A, b, d_in, d_out) + sub
    assert got == want
    z = faiss_io.parse_index(got)
    assert z["kind"] == "pretransform" and (z["d"], z["ntotal"]) == (d_in, 3)
    (t,) = z["chain"]
    np.testing.assert_array_equal(t["A"], A)
    assert (t["d_in"], t["d_out"], t["have_bias"]) == (d_in, d_out, bias)
    if bias:
        np.testing.assert_array_equal(t["b"], b)
    assert z["index"]["d"] == d_out
    for (i0, c0), (i1, c1) in zip(lists, z["index"]["lists"]):
        np.testing.assert_array_equal(i0, i1)
        np.testing.assert_array_equal(c0, c1)
    assert faiss_io.parse_index(sub)["kind"] == "ivfpq"


def test_pretransform_parse_errors(tmp_path):
    A = np.ones((8, 12), np.float32)
    sub, _ = _tiny_ivfpq(8)
    good = faiss_io.serialize_pretransform(12, 1, [(A, None, 12, 8, True)], sub, 3)
    p = tmp_path / "opq.index"
    p.write_bytes(good)
    assert faiss_io.is_faiss_file(p)
    with pytest.raises(RuntimeError, match="VectorTransform"):
        faiss_io.parse_index(good.replace(b"LTra", b"PcAm", 1))
    bad_dim = faiss_io.serialize_pretransform(12, 1, [(np.ones((6, 12), np.float32), None, 12, 6, True)], sub, 3)
    with pytest.raises(RuntimeError, match="output dimension"):
        faiss_io.parse_index(bad_dim)
    with pytest.raises(RuntimeError, match="truncated"):
        faiss_io.parse_index(good[:-5])
    with pytest.raises(RuntimeError, match="trailing"):
        faiss_io.parse_index(good + b"\0")


def test_vector_transform_file_roundtrip(tmp_path):
    rng = np.random.default_rng(6)
    lt = faiss.LinearTransform(10, 6, True)
    lt.set_matrix(rng.standard_normal((6, 10)), rng.standard_normal(6))
    p = tmp_path / "preproc.vectrans"
    faiss.write_VectorTransform(lt, p)
    assert p.read_bytes() == _ltra(lt.A, lt.b, 10, 6)
    back = faiss.read_VectorTransform(p)
    np.testing.assert_array_equal(back.A, lt.A)
    np.testing.assert_array_equal(back.b, lt.b)
    assert (back.d_in, back.d_out, back.is_trained) == (10, 6, True)
    assert faiss.downcast_VectorTransform(back) is back
