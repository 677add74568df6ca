"""Faiss IndexIVFPQ file layout (faiss_amd/faiss_io.py), CPU only.

Parity unpinned: no file written by real Faiss exists in the reference or the
image, so the byte layout is pinned by a field-by-field assembly of the upstream
Faiss 1.7.1 writer's order (index_write.cpp: write_index_header, write_ivf_header,
write_ProductQuantizer, write_InvertedLists), independent of the serializer."""
import struct

import numpy as np
import pytest

from faiss_amd import faiss_io


def _tiny(seed=0, sizes=(3, 2)):
    rng = np.random.default_rng(seed)
    d, M = 8, 2
    nlist = len(sizes)
    cent = rng.standard_normal((nlist, d)).astype(np.float32)
    cb = rng.standard_normal((M, 256, d // M)).astype(np.float32)
    lists = [(rng.integers(0, 1 << 40, n).astype(np.int64), rng.integers(0, 256, (n, M)).astype(np.uint8))
             for n in sizes]
    return d, nlist, M, cent, cb, lists


def _hand_assembled(d, nlist, nprobe, M, cent, cb, lists, kind):
    hdr = lambda dd, nt: struct.pack("<i", dd) + struct.pack("<q", nt) + struct.pack("<qq", 1 << 20, 1 << 20) \
        + struct.pack("<B", 1) + struct.pack("<i", 1)
    ntotal = sum(len(i) for i, _ in lists)
    b = b"IwPQ" + hdr(d, ntotal) + struct.pack("<Q", nlist) + struct.pack("<Q", nprobe)
    b += b"IxF2" + hdr(d, nlist) + struct.pack("<Q", cent.size) + cent.tobytes()
    b += struct.pack("<B", 0) + struct.pack("<Q", 0)                       # direct map: none, empty array
    b += struct.pack("<B", 1) + struct.pack("<Q", M)                       # by_residual, code_size
    b += struct.pack("<QQQ", d, M, 8) + struct.pack("<Q", cb.size) + cb.tobytes()
    b += b"ilar" + struct.pack("<QQ", nlist, M)
    sizes = [len(i) for i, _ in lists]
    if kind == "full":
        b += b"full" + struct.pack("<Q", nlist) + b"".join(struct.pack("<Q", n) for n in sizes)
    else:
        nz = [(l, n) for l, n in enumerate(sizes) if n]
        b += b"sprs" + struct.pack("<Q", 2 * len(nz)) + b"".join(struct.pack("<QQ", l, n) for l, n in nz)
    for ids, codes in lists:
        if len(ids):
            b += codes.tobytes() + ids.tobytes()
    return b


@pytest.mark.parametrize("sizes,kind", [((3, 2), "full"), ((4, 0, 0, 1), "sprs"), ((0, 5, 2), "full")])
def test_layout_matches_faiss_writer_order(sizes, kind):
    d, nlist, M, cent, cb, lists = _tiny(1, sizes)
    got = faiss_io.serialize_ivfpq(d, nlist, 7, M, 8, 1, cent, cb, lists)
    assert got == _hand_assembled(d, nlist, 7, M, cent, cb, lists, kind)


def test_parse_roundtrip():
    d, nlist, M, cent, cb, lists = _tiny(2, (5, 0, 3, 1))
    z = faiss_io.parse_ivfpq(faiss_io.serialize_ivfpq(d, nlist, 3, M, 8, 1, cent, cb, lists))
    assert (z["d"], z["nlist"], z["nprobe"], z["M"], z["nbits"], z["metric"]) == (d, nlist, 3, M, 8, 1)
    np.testing.assert_array_equal(z["centroids"], cent)
    np.testing.assert_array_equal(z["codebook"], cb)
    for (i0, c0), (i1, c1) in zip(lists, z["lists"]):
        np.testing.assert_array_equal(i0, i1)
        np.testing.assert_array_equal(c0, c1)


def test_parse_errors(tmp_path):
    d, nlist, M, cent, cb, lists = _tiny(3)
    buf = faiss_io.serialize_ivfpq(d, nlist, 1, M, 8, 1, cent, cb, lists)
    with pytest.raises(RuntimeError, match="truncated"):
        faiss_io.parse_ivfpq(buf[:-3])
    with pytest.raises(RuntimeError, match="fourcc"):
        faiss_io.parse_ivfpq(b"IxF2" + buf[4:])
    with pytest.raises(RuntimeError, match="legacy"):
        faiss_io.parse_ivfpq(b"IvPQ" + buf[4:])
    p = tmp_path / "x.index"
    p.write_bytes(buf)
    assert faiss_io.is_faiss_file(p)
    p.write_bytes(b"CHIVFPQ1" + buf)
    assert not faiss_io.is_faiss_file(p)
