"""Faiss binary index files for IndexIVFPQ.

Chameleon's harnesses persist trained/populated indexes with ``faiss.write_index``
and load them with ``faiss.read_index`` (``Chameleon/Faiss_experiments/
bench_polysemous_1bn.py:287, 290``; beir ``faiss_index.py:29``; the FPGA data
extraction reads such files, ``my_faiss_extract_scripts/extract_FPGA_required_data.py:
174-248``).  This module reads and writes that layout so those files move between
Faiss and faiss_amd unchanged.

The layout is restated from upstream Faiss 1.7.1 ``impl/index_write.cpp`` /
``index_read.cpp`` (not vendored in the reference, not installed here), little-endian:

    "IwPQ"                                   IndexIVFPQ (non-legacy inverted lists)
      index header: d i32, ntotal i64, 2 x dummy i64 (1 << 20), is_trained u8, metric_type i32
                    [metric_arg f32 if metric_type > 1]
      nlist u64, nprobe u64
      quantizer:   "IxF2" (L2) | "IxFI" (IP), index header, xb = u64 count + f32[count]
      direct map:  type u8 (0 = none), array = u64 count + i64[count]
      by_residual u8, code_size u64
      PQ:          d u64, M u64, nbits u64, centroids = u64 count + f32[count]   ([M][ksub][dsub])
      "ilar", nlist u64, code_size u64,
        "full" + u64 count + u64 sizes[nlist]   |   "sprs" + u64 count + u64 (list, size) pairs
        per non-empty list: codes u8[n * code_size], then ids i64[n]

    "IxPT"                                   IndexPreTransform (the OPQ front of "OPQ16,IVF..,PQ16")
      index header (d = the chain's d_in), nt i32, nt x VectorTransform, then the wrapped index
      VectorTransform "LTra" (LinearTransform, and OPQMatrix, which Faiss writes as a plain
      LinearTransform): have_bias u8, A = u64 count + f32[d_out * d_in], b = u64 count + f32[count],
      d_in i32, d_out i32, is_trained u8

Parity is unpinned: no Faiss-written file exists in the reference or this image
(the reference's ``*.index`` files are not shipped), so the tests check a
hand-assembled byte layout and round trips, not a file from real Faiss.
"""
from __future__ import annotations

import struct

import numpy as np

FOURCC_IVFPQ = b"IwPQ"
FOURCC_FLAT = {0: b"IxFI", 1: b"IxF2"}  # metric_type: 0 = INNER_PRODUCT, 1 = L2
HEADER_DUMMY = 1 << 20


FOURCC_PRETRANSFORM = b"IxPT"
FOURCC_LINEAR = b"LTra"


def is_faiss_file(path) -> bool:
    with open(path, "rb") as f:
        return f.read(4) in (FOURCC_IVFPQ, b"IvPQ", FOURCC_PRETRANSFORM)


class _Reader:
    def __init__(self, buf: bytes):
        self.b = memoryview(buf)
        self.o = 0

    def take(self, n):
        if self.o + n > len(self.b):
            raise RuntimeError("Faiss index file is truncated")
        v = self.b[self.o:self.o + n]
        self.o += n
        return v

    def fmt(self, f):
        return struct.unpack("<" + f, self.take(struct.calcsize("<" + f)))[0]

    def fourcc(self):
        return bytes(self.take(4))

    def vector(self, dtype):
        n = self.fmt("Q")
        it = np.dtype(dtype).itemsize
        return np.frombuffer(self.take(n * it), dtype=dtype).copy()

    def header(self):
        d = self.fmt("i")
        ntotal = self.fmt("q")
        self.fmt("q")
        self.fmt("q")
        is_trained = self.fmt("B") != 0
        metric = self.fmt("i")
        if metric > 1:
            self.fmt("f")
        return d, ntotal, is_trained, metric


def parse_ivfpq(buf: bytes) -> dict:
    """Faiss IndexIVFPQ bytes -> {d, nlist, nprobe, M, nbits, metric, is_trained,
    centroids [nlist][d], codebook [M][ksub][dsub], lists: [(ids i64[n], codes u8[n][code_size])]}."""
    r = _Reader(buf)
    z = _parse_ivfpq(r, r.fourcc())
    if r.o != len(r.b):
        raise RuntimeError("trailing bytes after the index")
    return z


def parse_index(buf: bytes) -> dict:
    """IndexIVFPQ or IndexPreTransform(LinearTransform..., IndexIVFPQ) bytes.
    IVF-PQ -> parse_ivfpq's dict with kind "ivfpq"; pre-transform -> {kind
    "pretransform", d, ntotal, metric, chain: [{A [d_out][d_in], b, have_bias,
    d_in, d_out, is_trained}], index: the IVF-PQ dict}."""
    r = _Reader(buf)
    h = r.fourcc()
    if h == FOURCC_PRETRANSFORM:
        d, ntotal, is_trained, metric = r.header()
        nt = r.fmt("i")
        chain = [_parse_linear(r) for _ in range(nt)]
        if not chain or chain[0]["d_in"] != d:
            raise RuntimeError("pre-transform chain does not match the index dimension")
        sub = _parse_ivfpq(r, r.fourcc())
        if sub["d"] != chain[-1]["d_out"]:
            raise RuntimeError("pre-transform output dimension does not match the wrapped index")
        z = {"kind": "pretransform", "d": d, "ntotal": ntotal, "metric": metric, "chain": chain, "index": sub}
    else:
        z = _parse_ivfpq(r, h)
    if r.o != len(r.b):
        raise RuntimeError("trailing bytes after the index")
    return z


def _parse_linear(r: _Reader) -> dict:
    vh = r.fourcc()
    if vh != FOURCC_LINEAR:
        raise RuntimeError(f"unsupported VectorTransform {vh!r} (LinearTransform / OPQMatrix only)")
    have_bias = r.fmt("B") != 0
    A = r.vector(np.float32)
    b = r.vector(np.float32)
    d_in = r.fmt("i")
    d_out = r.fmt("i")
    t_trained = r.fmt("B") != 0
    if t_trained and A.size != d_in * d_out:
        raise RuntimeError("LinearTransform matrix has the wrong size")
    if have_bias and t_trained and b.size != d_out:
        raise RuntimeError("LinearTransform bias has the wrong size")
    return {"A": A.reshape(d_out, d_in) if A.size else A, "b": b if have_bias else None,
            "have_bias": have_bias, "d_in": d_in, "d_out": d_out, "is_trained": t_trained}


def parse_vector_transform(buf: bytes) -> dict:
    """A faiss.write_VectorTransform file (bench_gpu_1bn.py:507-510): one "LTra" record."""
    r = _Reader(buf)
    t = _parse_linear(r)
    if r.o != len(r.b):
        raise RuntimeError("trailing bytes after the VectorTransform")
    return t


def serialize_linear(A, b, d_in, d_out, is_trained=True) -> bytes:
    A = np.zeros(0, np.float32) if A is None else np.ascontiguousarray(A, np.float32).reshape(-1)
    bb = np.zeros(0, np.float32) if b is None else np.ascontiguousarray(b, np.float32).reshape(-1)
    return b"".join([FOURCC_LINEAR, struct.pack("<B", 0 if b is None else 1), _vector(A), _vector(bb),
                     struct.pack("<iiB", d_in, d_out, 1 if is_trained else 0)])


def _parse_ivfpq(r: _Reader, h: bytes) -> dict:
    if h == b"IvPQ":
        raise RuntimeError("legacy IvPQ Faiss files (pre-1.5 inverted lists) are not supported")
    if h != FOURCC_IVFPQ:
        raise RuntimeError(f"not a Faiss IndexIVFPQ file (fourcc {h!r})")
    d, ntotal, is_trained, metric = r.header()
    nlist = r.fmt("Q")
    nprobe = r.fmt("Q")
    qh = r.fourcc()
    if qh not in (b"IxF2", b"IxFI"):
        raise RuntimeError(f"unsupported coarse quantizer {qh!r} (IndexFlatL2 / IndexFlatIP only)")
    qd, qn, _, _ = r.header()
    xb = r.vector(np.float32)
    if qd != d or xb.size != qn * d:
        raise RuntimeError("quantizer shape does not match the index")
    dm_type = r.fmt("B")
    dm = r.vector(np.int64)
    if dm_type != 0 or dm.size:
        raise RuntimeError("IVF direct maps are not supported")
    by_residual = r.fmt("B") != 0
    code_size = r.fmt("Q")
    pd = r.fmt("Q")
    M = r.fmt("Q")
    nbits = r.fmt("Q")
    cb = r.vector(np.float32)
    if not by_residual:
        raise RuntimeError("only by_residual IndexIVFPQ is supported")
    if pd != d or nbits != 8 or code_size != M or (is_trained and cb.size != M * 256 * (d // M)):
        raise RuntimeError("unsupported PQ shape (8-bit codes, code_size == M)")
    if r.fourcc() != b"ilar":
        raise RuntimeError("only ArrayInvertedLists ('ilar') are supported")
    il_n = r.fmt("Q")
    il_cs = r.fmt("Q")
    if il_n != nlist or il_cs != code_size:
        raise RuntimeError("inverted lists do not match the index")
    kind = r.fourcc()
    if kind == b"full":
        sizes = r.vector(np.uint64).astype(np.int64)
        if sizes.size != nlist:
            raise RuntimeError("inverted list size table has the wrong length")
    elif kind == b"sprs":
        pairs = r.vector(np.uint64).astype(np.int64).reshape(-1, 2)
        sizes = np.zeros(nlist, np.int64)
        sizes[pairs[:, 0]] = pairs[:, 1]
    else:
        raise RuntimeError(f"unknown inverted list size encoding {kind!r}")
    lists = []
    for l in range(nlist):
        n = int(sizes[l])
        if n:
            codes = np.frombuffer(r.take(n * code_size), np.uint8).reshape(n, code_size).copy()
            ids = np.frombuffer(r.take(n * 8), np.int64).copy()
        else:
            codes = np.zeros((0, code_size), np.uint8)
            ids = np.zeros(0, np.int64)
        lists.append((ids, codes))
    if int(sizes.sum()) != ntotal:
        raise RuntimeError("inverted list sizes do not add up to ntotal")
    return {"kind": "ivfpq", "d": d, "nlist": nlist, "nprobe": nprobe, "M": M, "nbits": nbits, "metric": metric,
            "is_trained": is_trained, "centroids": xb.reshape(nlist, d) if xb.size else xb,
            "codebook": cb.reshape(M, 256, d // M) if cb.size else cb, "lists": lists}


def _header(d, ntotal, is_trained, metric):
    return struct.pack("<iqqqBi", d, ntotal, HEADER_DUMMY, HEADER_DUMMY, 1 if is_trained else 0, metric)


def _vector(a):
    a = np.ascontiguousarray(a)
    return struct.pack("<Q", a.size) + a.tobytes()


def serialize_ivfpq(d, nlist, nprobe, M, nbits, metric, centroids, codebook, lists, is_trained=True) -> bytes:
    """The inverse of parse_ivfpq (sizes written as a "full" table, as Faiss does
    when more than half of the lists are non-empty, else "sprs")."""
    code_size = M * nbits // 8
    ntotal = sum(len(ids) for ids, _ in lists)
    cent = np.ascontiguousarray(centroids, np.float32).reshape(-1)
    out = [FOURCC_IVFPQ, _header(d, ntotal, is_trained, metric), struct.pack("<QQ", nlist, nprobe),
           FOURCC_FLAT[metric], _header(d, nlist if cent.size else 0, True, metric), _vector(cent),
           struct.pack("<B", 0), _vector(np.zeros(0, np.int64)),
           struct.pack("<BQ", 1, code_size), struct.pack("<QQQ", d, M, nbits),
           _vector(np.ascontiguousarray(codebook, np.float32).reshape(-1)),
           b"ilar", struct.pack("<QQ", nlist, code_size)]
    sizes = np.array([len(ids) for ids, _ in lists], np.uint64)
    nz = np.nonzero(sizes)[0]
    if len(nz) > nlist // 2:
        out += [b"full", _vector(sizes)]
    else:
        out += [b"sprs", _vector(np.stack([nz.astype(np.uint64), sizes[nz]], 1).reshape(-1))]
    for ids, codes in lists:
        if len(ids):
            out.append(np.ascontiguousarray(codes, np.uint8).tobytes())
            out.append(np.ascontiguousarray(ids, np.int64).tobytes())
    return b"".join(out)


def serialize_pretransform(d, metric, chain, sub: bytes, ntotal, is_trained=True) -> bytes:
    """IndexPreTransform bytes: chain = [(A [d_out][d_in] | None, b | None, d_in, d_out, is_trained)],
    sub = the wrapped index's bytes (serialize_ivfpq)."""
    out = [FOURCC_PRETRANSFORM, _header(d, ntotal, is_trained, metric), struct.pack("<i", len(chain))]
    out += [serialize_linear(*t) for t in chain]
    out.append(sub)
    return b"".join(out)
