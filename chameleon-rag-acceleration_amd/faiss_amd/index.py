"""Faiss-compatible index classes backed by the gfx950 engine (libivfpq.so).

The surface mirrors what Chameleon's callers use on ``faiss`` (SURVEY.md
§8(b)):

* ``IndexIVFPQ(quantizer, d, nlist, M, nbits)`` with ``train / add /
  add_with_ids / search / search_preassigned / reset``, ``nprobe``,
  ``ntotal``, ``d``, ``is_trained``, ``quantizer``, ``pq.centroids``,
  ``invlists.{list_size,get_ids,get_codes,imbalance_factor}``,
  ``precomputed_table``, ``parallel_mode``
  (``bench_polysemous_1bn.py:272-291, 343-345, 368, 422, 430``;
  ``beir/beir/retrieval/search/dense/faiss_index.py:13-96``;
  ``ralm/retriever/faiss_retriever.py:18-275``;
  ``my_faiss_extract_scripts/extract_FPGA_required_data.py:174-248``);
* ``IndexFlatL2`` (the coarse quantizer; exact search on the GPU);
* ``index_factory``, ``ParameterSpace``, ``read_index / write_index``,
  ``swig_ptr``, ``vector_to_array``, ``get_num_gpus``.

Numpy conventions as Faiss: float32 C-contiguous in; ``D`` float32 and ``I``
int64 out; missing results are (FLT_MAX, -1).  Errors raise ``RuntimeError``
(Faiss's SWIG layer turns ``FaissException`` into ``RuntimeError`` too).
"""
from __future__ import annotations

import ctypes
import re

import numpy as np

from . import _lib, faiss_io

METRIC_INNER_PRODUCT = 0
METRIC_L2 = 1
MAX_K = 1024


def _f32(x, d=None, name="x"):
    a = np.ascontiguousarray(x, dtype=np.float32)
    if a.ndim != 2 or (d is not None and a.shape[1] != d):
        raise RuntimeError(f"{name} must be a float32 matrix with {d} columns, got shape {a.shape}")
    return a


def _ptr(a, t):
    return a.ctypes.data_as(t)


def swig_ptr(a):
    """Faiss passes raw pointers to the 8-argument search_preassigned; here the
    array itself is passed through (faiss_retriever.py:217-223)."""
    return a


def vector_to_array(v):
    return np.asarray(v).copy()


def downcast_index(index):
    """faiss.downcast_index: Python objects already have their concrete type."""
    return index


def extract_index_ivf(index):
    """faiss.extract_index_ivf: the IndexIVFPQ inside an IndexPreTransform."""
    return getattr(index, "index", index)


def get_num_gpus():
    return int(_lib.load().ivfpq_device_count())


def _default_device():
    try:
        import torch

        if torch.cuda.is_available():
            return torch.cuda.current_device()
    except Exception:
        pass
    return 0


class IndexFlatL2:
    """Exact L2 search (faiss.IndexFlatL2).  As an IVF quantizer it holds the
    coarse centroids (``quantizer.xb``, extract_FPGA_required_data.py:174-184);
    standalone, ``search`` runs the GPU distance + select kernels (the
    IndexScanner coarse service, ralm/index_scanner/index_scanner.py:61-77)."""

    metric_type = METRIC_L2
    is_trained = True

    def __init__(self, d, device=None):
        self.d = d
        self.device = _default_device() if device is None else device
        self._xb = np.zeros((0, d), np.float32)

    @property
    def ntotal(self):
        return self._xb.shape[0]

    @property
    def xb(self):
        return self._xb.reshape(-1)

    def add(self, x):
        x = _f32(x, self.d)
        self._xb = np.concatenate([self._xb, x]) if self.ntotal else x.copy()

    def reset(self):
        self._xb = np.zeros((0, self.d), np.float32)

    def reconstruct(self, i):
        return self._xb[i].copy()

    def reconstruct_n(self, i0, n):
        return self._xb[i0:i0 + n].copy()

    def train(self, x):
        pass

    def search(self, x, k):
        x = _f32(x, self.d)
        n = x.shape[0]
        if not 1 <= k <= MAX_K:
            raise RuntimeError(f"k must be in [1, {MAX_K}]")
        D = np.empty((n, k), np.float32)
        I = np.empty((n, k), np.int64)
        L = _lib.load()
        _lib.check(L.ivfpq_flat_search(self.device, self.d, self.ntotal, _ptr(self._xb, _lib.c_f32p), n,
                                       _ptr(x, _lib.c_f32p), k, self.metric_type, _ptr(D, _lib.c_f32p),
                                       _ptr(I, _lib.c_i64p)))
        return D, I


class IndexFlatIP(IndexFlatL2):
    """Exact inner-product search (faiss.IndexFlatIP): the quantizer of an
    inner-product IndexIVFPQ and beir's flat IP index
    (beir/beir/retrieval/search/dense/faiss_search.py:14-131).  Results are the
    k largest inner products, descending."""

    metric_type = METRIC_INNER_PRODUCT


class _ProductQuantizer:
    """index.pq view: M, nbits, ksub, dsub and ``centroids`` (M*256*dsub floats,
    the layout of faiss pq.centroids)."""

    def __init__(self, owner):
        self._o = owner

    M = property(lambda self: self._o.M)
    nbits = property(lambda self: self._o.nbits)
    ksub = property(lambda self: 1 << self._o.nbits)
    dsub = property(lambda self: self._o.d // self._o.M)
    code_size = property(lambda self: self._o.M * self._o.nbits // 8)

    @property
    def centroids(self):
        return self._o.codebook().reshape(-1)

    def get_centroids(self, m, j):
        return self._o.codebook()[m, j].copy()


class _InvertedLists:
    """index.invlists view (faiss ArrayInvertedLists read API)."""

    def __init__(self, owner):
        self._o = owner

    @property
    def nlist(self):
        return self._o.nlist

    @property
    def code_size(self):
        return self._o.M

    def list_sizes(self):
        out = np.empty(self._o.nlist, np.int64)
        _lib.check(_lib.load().ivfpq_get_list_sizes(self._o._h, _ptr(out, _lib.c_i64p)))
        return out

    def list_size(self, l):
        return int(self.list_sizes()[l])

    def _get(self, l):
        n = self.list_size(l)
        codes = np.empty((n, self._o.M), np.uint8)
        ids = np.empty(n, np.int64)
        _lib.check(_lib.load().ivfpq_get_list(self._o._h, int(l), _ptr(codes, _lib.c_u8p),
                                              _ptr(ids, _lib.c_i64p)))
        return codes, ids

    def get_codes(self, l):
        return self._get(l)[0].reshape(-1)

    def export(self):
        """All lists at once: (list_no int64 [ntotal], codes uint8 [ntotal][M], ids
        int64 [ntotal]) in list order (each list in its stored order), the input of
        add_preencoded -- one list-size query instead of one per list."""
        sizes = self.list_sizes()
        tot = int(sizes.sum())
        codes = np.empty((tot, self._o.M), np.uint8)
        ids = np.empty(tot, np.int64)
        off = np.concatenate([[0], np.cumsum(sizes)])
        L = _lib.load()
        for l in np.nonzero(sizes)[0]:
            _lib.check(L.ivfpq_get_list(self._o._h, int(l), _ptr(codes[off[l]:], _lib.c_u8p),
                                        _ptr(ids[off[l]:], _lib.c_i64p)))
        return np.repeat(np.arange(self._o.nlist, dtype=np.int64), sizes), codes, ids

    def get_ids(self, l):
        return self._get(l)[1]

    def imbalance_factor(self):
        """faiss InvertedLists::imbalance_factor: nlist * sum(n_l^2) / ntotal^2."""
        s = self.list_sizes().astype(np.float64)
        tot = s.sum()
        return float(len(s) * (s * s).sum() / (tot * tot)) if tot else 0.0



def overlap_built():
    """True: the batches-in-flight overlap is available (ivfpq_overlap_built; kept
    for callers of the r04 interface, where it was a build option)."""
    return bool(_lib.load().ivfpq_overlap_built())

class IndexIVFPQ:
    """faiss.IndexIVFPQ (by_residual; METRIC_L2 with precomputed tables, or
    METRIC_INNER_PRODUCT) on one MI355X."""

    by_residual = True
    use_precomputed_table = 1
    polysemous_ht = 0

    def __init__(self, quantizer, d, nlist, M, nbits=8, metric=METRIC_L2, device=None, _handle=None):
        self.d = int(d)
        self.nlist = int(nlist)
        self.M = int(M)
        self.nbits = int(nbits)
        self.metric_type = metric
        self.device = _default_device() if device is None else int(device)
        if quantizer is None:
            quantizer = (IndexFlatIP if metric == METRIC_INNER_PRODUCT else IndexFlatL2)(d, self.device)
        self.quantizer = quantizer
        self.parallel_mode = 0  # accepted for faiss_retriever.py:71; queries are always independent
        self.verbose = False
        self.niter_coarse = 25
        self.niter_pq = 25
        self.seed = 1234
        L = _lib.load()
        if _handle is not None:
            self._h = _handle
        else:
            h = _lib.c_handle()
            _lib.check(L.ivfpq_create(self.d, self.nlist, self.M, self.nbits, metric, self.device, ctypes.byref(h)))
            self._h = h
        self.pq = _ProductQuantizer(self)
        self.invlists = _InvertedLists(self)
        self._codebook_cache = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib._lib is not None:
            _lib._lib.ivfpq_free(h)
            self._h = None

    # ------------------------------------------------------------ properties
    @property
    def ntotal(self):
        return int(_lib.load().ivfpq_ntotal(self._h))

    @property
    def is_trained(self):
        return bool(_lib.load().ivfpq_is_trained(self._h))

    @property
    def nprobe(self):
        return int(_lib.load().ivfpq_get_nprobe(self._h))

    @nprobe.setter
    def nprobe(self, p):
        _lib.check(_lib.load().ivfpq_set_nprobe(self._h, int(p)))

    @property
    def code_size(self):
        return self.M

    def codebook(self):
        if self._codebook_cache is None:
            cb = np.empty((self.M, 1 << self.nbits, self.d // self.M), np.float32)
            _lib.check(_lib.load().ivfpq_get_codebook(self._h, _ptr(cb, _lib.c_f32p)))
            self._codebook_cache = cb
        return self._codebook_cache

    def centroids(self):
        c = np.empty((self.nlist, self.d), np.float32)
        _lib.check(_lib.load().ivfpq_get_centroids(self._h, _ptr(c, _lib.c_f32p)))
        return c

    @property
    def precomputed_table(self):
        t = np.empty((self.nlist, self.M, 1 << self.nbits), np.float32)
        _lib.check(_lib.load().ivfpq_get_precomputed_table(self._h, _ptr(t, _lib.c_f32p)))
        return t.reshape(-1)

    def _sync_quantizer(self):
        if isinstance(self.quantizer, IndexFlatL2):  # IndexFlatIP too
            self.quantizer.reset()
            self.quantizer.add(self.centroids())

    # ----------------------------------------------------------- build path
    def train(self, x):
        x = _f32(x, self.d)
        _lib.check(_lib.load().ivfpq_train(self._h, x.shape[0], _ptr(x, _lib.c_f32p), self.niter_coarse,
                                           self.niter_pq, self.seed))
        self._codebook_cache = None
        self._sync_quantizer()

    def set_trained(self, centroids, codebook):
        """Install trained quantizers (coarse centroids [nlist][d], PQ codebook [M][256][d/M])."""
        c = _f32(np.asarray(centroids).reshape(self.nlist, self.d), self.d, "centroids")
        cb = np.ascontiguousarray(codebook, np.float32).reshape(-1)
        if cb.size != self.M * (1 << self.nbits) * (self.d // self.M):
            raise RuntimeError("codebook has the wrong size")
        _lib.check(_lib.load().ivfpq_set_trained(self._h, _ptr(c, _lib.c_f32p), _ptr(cb, _lib.c_f32p)))
        self._codebook_cache = None
        self._sync_quantizer()

    def add(self, x):
        x = _f32(x, self.d)
        _lib.check(_lib.load().ivfpq_add(self._h, x.shape[0], _ptr(x, _lib.c_f32p), None))

    def add_with_ids(self, x, ids):
        x = _f32(x, self.d)
        ids = np.ascontiguousarray(ids, np.int64).reshape(-1)
        if ids.shape[0] != x.shape[0]:
            raise RuntimeError("ids and x have different lengths")
        _lib.check(_lib.load().ivfpq_add(self._h, x.shape[0], _ptr(x, _lib.c_f32p), _ptr(ids, _lib.c_i64p)))

    def add_preencoded(self, list_no, codes, ids=None):
        list_no = np.ascontiguousarray(list_no, np.int64).reshape(-1)
        codes = np.ascontiguousarray(codes, np.uint8).reshape(-1, self.M)
        n = list_no.shape[0]
        if codes.shape[0] != n:
            raise RuntimeError("codes and list_no have different lengths")
        idp = None
        if ids is not None:
            ids = np.ascontiguousarray(ids, np.int64).reshape(-1)
            idp = _ptr(ids, _lib.c_i64p)
        _lib.check(_lib.load().ivfpq_add_preencoded(self._h, n, _ptr(list_no, _lib.c_i64p),
                                                    _ptr(codes, _lib.c_u8p), idp))

    def reset(self):
        _lib.check(_lib.load().ivfpq_reset(self._h))

    def set_list_range(self, lo, hi):
        """Keep and scan only inverted lists [lo, hi) (list-range sharding)."""
        _lib.check(_lib.load().ivfpq_set_list_range(self._h, int(lo), int(hi)))

    # ------------------------------------------------------------ search path
    def _check_k(self, k):
        if not 1 <= int(k) <= MAX_K:
            raise RuntimeError(f"k must be in [1, {MAX_K}], got {k}")

    def search(self, x, k):
        x = _f32(x, self.d)
        self._check_k(k)
        n = x.shape[0]
        D = np.empty((n, k), np.float32)
        I = np.empty((n, k), np.int64)
        _lib.check(_lib.load().ivfpq_search(self._h, n, _ptr(x, _lib.c_f32p), int(k), _ptr(D, _lib.c_f32p),
                                            _ptr(I, _lib.c_i64p)))
        return D, I

    def search_preassigned(self, *args):
        """Either ``search_preassigned(x, k, Iq, Dq=None) -> (D, I)`` or the
        Faiss C++ form ``search_preassigned(n, x, k, Iq, Dq, D, I, store_pairs)``
        that fills D and I (faiss_retriever.py:217-223)."""
        if len(args) >= 7:
            n, x, k, Iq, Dq, D, I = args[:7]
            if len(args) > 7 and args[7]:
                raise RuntimeError("store_pairs is not supported")
            Dr, Ir = self._search_preassigned(x, k, Iq, Dq)
            np.copyto(np.asarray(D).reshape(Dr.shape), Dr)
            np.copyto(np.asarray(I).reshape(Ir.shape), Ir)
            return None
        x, k, Iq = args[:3]
        Dq = args[3] if len(args) > 3 else None
        return self._search_preassigned(x, k, Iq, Dq)

    def _search_preassigned(self, x, k, Iq, Dq=None):
        x = _f32(np.asarray(x).reshape(-1, self.d), self.d)
        self._check_k(k)
        n = x.shape[0]
        Iq = np.ascontiguousarray(Iq, np.int64).reshape(n, -1)
        if Iq.shape[1] != self.nprobe:
            raise RuntimeError(f"Iq must have nprobe={self.nprobe} columns, got {Iq.shape[1]}")
        Dqp = None
        if Dq is not None:
            Dq = np.ascontiguousarray(Dq, np.float32).reshape(Iq.shape)
            Dqp = _ptr(Dq, _lib.c_f32p)
        D = np.empty((n, k), np.float32)
        I = np.empty((n, k), np.int64)
        _lib.check(_lib.load().ivfpq_search_preassigned(self._h, n, _ptr(x, _lib.c_f32p), int(k),
                                                        _ptr(Iq, _lib.c_i64p), Dqp, _ptr(D, _lib.c_f32p),
                                                        _ptr(I, _lib.c_i64p)))
        return D, I

    def serve_request(self, msg, batch_size, dim, with_lists=False, nprobe=None, out=None):
        """One FaissServer request (RALM wire format, ``faiss_amd.wire``) in, the
        encoded answer out: decode + search (or search_preassigned) + encode in
        one native call (``ivfpq_serve_request``).  ``out``: optional writable
        buffer of at least ``answer_message_len(k, batch_size)`` bytes, filled
        in place; returns the answer as ``bytearray`` (or ``out``'s view)."""
        buf = np.frombuffer(msg, np.uint8)
        np_ = int(self.nprobe if nprobe is None else nprobe)
        if out is None:
            from .wire import peek_k

            k = peek_k(msg, with_lists)
            out = bytearray(max(1, batch_size * k * 12))
        ans = np.frombuffer(out, np.uint8)
        if not ans.flags.writeable:
            raise RuntimeError("answer buffer must be writable")
        ln = ctypes.c_int64(0)
        # a plain request is searched with the index's nprobe: an explicit nprobe
        # applies for this call only (with lists, it is the request's column count)
        saved = self.nprobe
        if not with_lists and nprobe is not None:
            self.nprobe = np_
        try:
            _lib.check(_lib.load().ivfpq_serve_request(self._h, _ptr(buf, _lib.c_u8p), buf.size,
                                                       int(bool(with_lists)), int(batch_size), int(dim), np_,
                                                       _ptr(ans, _lib.c_u8p), ans.size, ctypes.byref(ln)))
        finally:
            if self.nprobe != saved:
                self.nprobe = saved
        return out if len(out) == ln.value else memoryview(out)[:ln.value]

    # ------------------------------------------------------------ stage timing
    STAGES = ("coarse", "tables", "scan", "lists")

    def set_timing(self, on=True, lists_only=False):
        """Record HIP events around every stage (or, lists_only, around the list-scan kernel alone)."""
        _lib.check(_lib.load().ivfpq_set_timing(self._h, (2 if lists_only else 1) if on else 0))

    def get_timing(self):
        """{stage: (total_ms, launches)} since the last call (waits for the events)."""
        ms = (ctypes.c_double * len(self.STAGES))()
        cnt = (ctypes.c_int64 * len(self.STAGES))()
        _lib.check(_lib.load().ivfpq_get_timing(self._h, ms, cnt))
        return {s: (ms[i], cnt[i]) for i, s in enumerate(self.STAGES)}

    # ------------------------------------------------- device (torch) entry points
    def _check_dev(self, t, name, dtype, shape):
        """The C-ABI takes raw device pointers: anything but a contiguous tensor of
        the exact dtype and shape on this index's device would be read or written
        out of bounds, so it is rejected here (as the host path rejects bad arrays)."""
        import torch

        if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
            raise RuntimeError(f"{name} must be a CUDA tensor")
        if t.device.index != self.device:
            raise RuntimeError(f"{name} is on cuda:{t.device.index}, the index on cuda:{self.device}")
        if t.dtype != dtype:
            raise RuntimeError(f"{name} must be {dtype}, got {t.dtype}")
        if tuple(t.shape) != tuple(shape):
            raise RuntimeError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
        if not t.is_contiguous():
            raise RuntimeError(f"{name} must be contiguous")
        return t

    def _dev_outputs(self, x, k, D, I):
        import torch

        n = x.shape[0]
        if D is None:
            D = torch.empty((n, k), dtype=torch.float32, device=x.device)
        if I is None:
            I = torch.empty((n, k), dtype=torch.int64, device=x.device)
        self._check_dev(D, "D", torch.float32, (n, k))
        self._check_dev(I, "I", torch.int64, (n, k))
        return D, I

    def _stream(self, x, stream):
        import torch

        return stream if stream is not None else torch.cuda.current_stream(x.device).cuda_stream

    @property
    def inflight(self):
        """Batches in flight: True lets device searches issued on different
        streams overlap (each stream keeps its own workspace, up to three);
        False (default, unless IVFPQ_INFLIGHT=1 at creation) orders each search
        after those still in flight on other streams.  Results are the same in
        both modes (tests/test_gpu_parity.py
        test_batches_in_flight_stress)."""
        return bool(_lib.load().ivfpq_get_inflight(self._h))

    @inflight.setter
    def inflight(self, on):
        _lib.check(_lib.load().ivfpq_set_inflight(self._h, int(bool(on))))

    def error_count(self):
        """Index-check violations counted by the merge kernels since creation
        (ivfpq_get_error_count; 0 on a correct run).  Waits for in-flight searches."""
        out = ctypes.c_int64(0)
        _lib.check(_lib.load().ivfpq_get_error_count(self._h, ctypes.byref(out)))
        return out.value

    def repair_stats(self):
        """(stale_reads, repairs) since creation: (query, merge launch) pairs that read a
        partial-list entry this batch's scan did not leave there, and the probes the merge
        rescanned because of one (ivfpq_get_repair_stats).  Waits for in-flight searches."""
        st, rp = ctypes.c_int64(0), ctypes.c_int64(0)
        _lib.check(_lib.load().ivfpq_get_repair_stats(self._h, ctypes.byref(st), ctypes.byref(rp)))
        return st.value, rp.value

    def repair_log(self, max_events=192):
        """The first stale-entry events as dicts (ivfpq_get_repair_log)."""
        buf = (ctypes.c_uint32 * (8 * max_events))()
        n = ctypes.c_int(0)
        _lib.check(_lib.load().ivfpq_get_repair_log(self._h, buf, int(max_events), ctypes.byref(n)))
        out = []
        for e in range(n.value):
            w = buf[8 * e:8 * e + 8]
            out.append({"site": w[0] & 0xFF, "reader_xcd": (w[0] >> 8) & 0xF, "query": w[1], "list": w[2] & 0xFFFF,
                         "rank": w[2] >> 16, "expected_tag": w[3], "found_tag": w[4] & 0x0FFFFFFF,
                         "writer_xcd": w[4] >> 28, "found_key_bits": w[5], "epoch": w[6], "reread": w[7]})
        return out

    def set_fault_injection(self, every):
        """Test hook: later searches skip the partial-list stores of slots with
        slot % every == 1 (0 = off); results must stay exact (repairs)."""
        _lib.check(_lib.load().ivfpq_set_fault_injection(self._h, int(every)))

    def search_device(self, x, k, D=None, I=None, stream=None):
        """Search with inputs resident in HBM.  ``x`` is a torch float32 CUDA
        tensor [n, d] on the index's device; returns torch (D, I) there, launched
        on ``stream`` (default: torch's current stream).  Searches of one index
        may be issued on different streams without synchronizing: the library
        orders each search after those still in flight on other streams, or,
        with ``inflight`` on, lets them overlap."""
        import torch

        self._check_k(k)
        self._check_dev(x, "x", torch.float32, (x.shape[0] if x.dim() == 2 else -1, self.d))
        D, I = self._dev_outputs(x, k, D, I)
        _lib.check(_lib.load().ivfpq_search_device(self._h, x.shape[0], x.data_ptr(), int(k), D.data_ptr(),
                                                   I.data_ptr(), ctypes.c_void_p(self._stream(x, stream))))
        return D, I

    def search_preassigned_device(self, x, k, Iq, Dq=None, D=None, I=None, stream=None, tables=None):
        """search_preassigned with HBM-resident inputs.  ``tables``: the token of a
        ``precompute_tables_device(x)`` call for exactly these queries, whose T3
        this search consumes instead of building its own."""
        import torch

        self._check_k(k)
        n = x.shape[0] if x.dim() == 2 else -1
        self._check_dev(x, "x", torch.float32, (n, self.d))
        self._check_dev(Iq, "Iq", torch.int64, (n, self.nprobe))
        if Dq is not None:
            self._check_dev(Dq, "Dq", torch.float32, (n, self.nprobe))
        D, I = self._dev_outputs(x, k, D, I)
        if tables is not None:
            _lib.check(_lib.load().ivfpq_search_preassigned_tables_device(
                self._h, n, x.data_ptr(), int(k), Iq.data_ptr(), Dq.data_ptr() if Dq is not None else None,
                D.data_ptr(), I.data_ptr(), ctypes.c_uint64(int(tables)), ctypes.c_void_p(self._stream(x, stream))))
        else:
            _lib.check(_lib.load().ivfpq_search_preassigned_device(
                self._h, n, x.data_ptr(), int(k), Iq.data_ptr(), Dq.data_ptr() if Dq is not None else None,
                D.data_ptr(), I.data_ptr(), ctypes.c_void_p(self._stream(x, stream))))
        return D, I

    def precompute_tables_device(self, x, stream=None):
        """T3 of the queries x (torch CUDA [n, d]) on ``stream``; returns the token
        that ``search_preassigned_device(x, ..., tables=token)`` consumes.  The
        shard flow runs it on a side stream while the coarse step and the probe
        all-gather run.  Up to three tokens can be pending."""
        import torch

        n = x.shape[0] if x.dim() == 2 else -1
        self._check_dev(x, "x", torch.float32, (n, self.d))
        tok = ctypes.c_uint64(0)
        _lib.check(_lib.load().ivfpq_precompute_tables_device(self._h, n, x.data_ptr(),
                                                              ctypes.c_void_p(self._stream(x, stream)),
                                                              ctypes.byref(tok)))
        return tok.value

    def add_device(self, x, ids=None, stream=None):
        """add / add_with_ids with the vectors already in HBM (torch float32 CUDA
        tensor [n, d]; ids: int64 CUDA tensor [n] or None for sequential ids).
        Assignment, encoding and the list-image merge run on the GPU; returns
        once the new image is in place."""
        import torch

        n = x.shape[0] if x.dim() == 2 else -1
        self._check_dev(x, "x", torch.float32, (n, self.d))
        if ids is not None:
            self._check_dev(ids, "ids", torch.int64, (n,))
        _lib.check(_lib.load().ivfpq_add_device(self._h, n, x.data_ptr(), ids.data_ptr() if ids is not None else None,
                                                ctypes.c_void_p(self._stream(x, stream))))

    def coarse_device(self, x, Iq=None, Dq=None, stream=None):
        """The coarse quantizer alone: (Dq, Iq) [n, min(nprobe, nlist)] -- L2
        distances ascending or inner products descending."""
        import torch

        n = x.shape[0] if x.dim() == 2 else -1
        self._check_dev(x, "x", torch.float32, (n, self.d))
        p = min(self.nprobe, self.nlist)
        if Iq is None:
            Iq = torch.empty((n, p), dtype=torch.int64, device=x.device)
        if Dq is None:
            Dq = torch.empty((n, p), dtype=torch.float32, device=x.device)
        self._check_dev(Iq, "Iq", torch.int64, (n, p))
        self._check_dev(Dq, "Dq", torch.float32, (n, p))
        _lib.check(_lib.load().ivfpq_coarse_device(self._h, n, x.data_ptr(), Iq.data_ptr(), Dq.data_ptr(),
                                                   ctypes.c_void_p(self._stream(x, stream))))
        return Dq, Iq

    def coarse_tables_device(self, x, x_tables, Iq=None, Dq=None, stream=None):
        """The list-range shard step's front half on one stream: the coarse quantizer
        of this rank's queries ``x`` and T3 of the global batch ``x_tables`` (one
        launch at nlist < 8192).  Returns (Dq, Iq, token); the token goes to
        ``search_preassigned_device(x_tables, ..., tables=token)``."""
        import torch

        n = x.shape[0] if x.dim() == 2 else -1
        self._check_dev(x, "x", torch.float32, (n, self.d))
        nt = x_tables.shape[0] if x_tables.dim() == 2 else -1
        self._check_dev(x_tables, "x_tables", torch.float32, (nt, self.d))
        p = min(self.nprobe, self.nlist)
        if Iq is None:
            Iq = torch.empty((n, p), dtype=torch.int64, device=x.device)
        if Dq is None:
            Dq = torch.empty((n, p), dtype=torch.float32, device=x.device)
        self._check_dev(Iq, "Iq", torch.int64, (n, p))
        self._check_dev(Dq, "Dq", torch.float32, (n, p))
        tok = ctypes.c_uint64(0)
        _lib.check(_lib.load().ivfpq_coarse_tables_device(self._h, n, x.data_ptr(), Iq.data_ptr(), Dq.data_ptr(), nt,
                                                          x_tables.data_ptr(), ctypes.c_void_p(self._stream(x, stream)),
                                                          ctypes.byref(tok)))
        return Dq, Iq, tok.value


def merge_topk_device(Ds, Is, metric=METRIC_L2, stream=None):
    """Merge S sorted partial results (torch [S, n, k]) into [n, k] on the GPU:
    ascending L2 distances, or descending inner products (metric)."""
    import torch

    if Ds.dim() != 3 or Is.shape != Ds.shape or Ds.dtype != torch.float32 or Is.dtype != torch.int64:
        raise RuntimeError("merge_topk_device: Ds float32 [S, n, k] and Is int64 of the same shape")
    if not (Ds.is_cuda and Is.is_cuda and Ds.device == Is.device):
        raise RuntimeError("merge_topk_device: inputs must be on one CUDA device")
    Ds, Is = Ds.contiguous(), Is.contiguous()
    S, n, k = Ds.shape
    D = torch.empty((n, k), dtype=torch.float32, device=Ds.device)
    I = torch.empty((n, k), dtype=torch.int64, device=Ds.device)
    s = stream if stream is not None else torch.cuda.current_stream(Ds.device).cuda_stream
    _lib.check(_lib.load().ivfpq_merge_topk_device(S, n, k, int(metric), Ds.data_ptr(), Is.data_ptr(),
                                                   D.data_ptr(), I.data_ptr(), ctypes.c_void_p(s)))
    return D, I


# ------------------------------------------------------------------ factory / IO

_FACTORY_RE = re.compile(r"^(?:OPQ(\d+)(?:_(\d+))?,)?IVF(\d+),PQ(\d+)(?:x(\d+))?$")


def parse_factory(key):
    """'[OPQ<M>[_<dout>],]IVF<nlist>,PQ<M>[x8]' -> (nlist, M, nbits) or, with an
    OPQ front, (nlist, M, nbits, opq_M, opq_dout) (opq_dout = -1: d)."""
    m = _FACTORY_RE.match(key.replace(" ", ""))
    if not m:
        raise RuntimeError(f"index_factory: unsupported key {key!r} "
                           "(supported: '[OPQ<M>[_<dout>],]IVF<nlist>,PQ<M>[x8]')")
    nbits = int(m.group(5)) if m.group(5) else 8
    base = (int(m.group(3)), int(m.group(4)), nbits)
    if m.group(1) is None:
        return base
    return base + (int(m.group(1)), int(m.group(2)) if m.group(2) else -1)


def index_factory(d, key, metric=METRIC_L2, device=None):
    """faiss.index_factory(d, "IVF1024,PQ16") (bench_polysemous_1bn.py:272) and the
    OPQ-fronted "OPQ16,IVF262144,PQ16" (bench_gpu_1bn.py:10-17)."""
    from .transform import IndexPreTransform, OPQMatrix

    f = parse_factory(key)
    if len(f) == 3:
        nlist, M, nbits = f
        return IndexIVFPQ(None, d, nlist, M, nbits, metric, device)
    nlist, M, nbits, opq_M, opq_dout = f
    opq = OPQMatrix(d, opq_M, opq_dout)
    return IndexPreTransform(opq, IndexIVFPQ(None, opq.d_out, nlist, M, nbits, metric, device))


class ParameterSpace:
    """faiss.ParameterSpace subset: set_index_parameters(index, "nprobe=16")."""

    def initialize(self, index):
        pass

    def set_index_parameter(self, index, name, value):
        if name != "nprobe":
            raise RuntimeError(f"unsupported parameter {name}")
        index.nprobe = int(value)

    def set_index_parameters(self, index, params):
        for kv in params.split(","):
            if not kv:
                continue
            name, value = kv.split("=")
            self.set_index_parameter(index, name.strip(), float(value))


def _ivfpq_bytes(index):
    inv = index.invlists
    lists = [(inv.get_ids(l), inv.get_codes(l).reshape(-1, index.code_size)) for l in range(index.nlist)]
    return faiss_io.serialize_ivfpq(index.d, index.nlist, index.nprobe, index.M, index.nbits, index.metric_type,
                                    index.centroids(), index.codebook(), lists)


def write_index(index, path, fmt="faiss"):
    """Persist ``index``.  fmt "faiss": the Faiss 1.7.1 IndexIVFPQ / IndexPreTransform
    binary layout (``faiss.read_index`` loads it; faiss_io.py); "native": this
    library's CHIVFPQ1 image (also keeps untrained indexes; IVF-PQ only)."""
    from .transform import IndexPreTransform

    if isinstance(index, IndexPreTransform):
        if fmt != "faiss" or not index.is_trained:
            raise RuntimeError("IndexPreTransform is written in the Faiss layout once trained")
        chain = [(t.A, t.b, t.d_in, t.d_out, t.is_trained) for t in index.chain]
        buf = faiss_io.serialize_pretransform(index.d, index.metric_type, chain, _ivfpq_bytes(index.index),
                                              index.ntotal)
    elif fmt == "native" or not index.is_trained:
        _lib.check(_lib.load().ivfpq_save(index._h, str(path).encode()))
        return
    elif fmt != "faiss":
        raise RuntimeError(f"unknown index file format {fmt!r}")
    else:
        buf = _ivfpq_bytes(index)
    with open(path, "wb") as f:
        f.write(buf)


def _ivfpq_from_dict(z, device):
    idx = IndexIVFPQ(None, z["d"], z["nlist"], z["M"], z["nbits"], z["metric"], device)
    if z["is_trained"]:
        idx.set_trained(z["centroids"], z["codebook"])
        nonempty = [(l, ids, codes) for l, (ids, codes) in enumerate(z["lists"]) if len(ids)]
        if nonempty:
            idx.add_preencoded(np.concatenate([np.full(len(ids), l, np.int64) for l, ids, _ in nonempty]),
                               np.concatenate([codes for _, _, codes in nonempty]),
                               np.concatenate([ids for _, ids, _ in nonempty]))
    idx.nprobe = max(1, min(int(z["nprobe"]), z["nlist"]))
    return idx


def read_index(path, device=None):
    """Load a Faiss IndexIVFPQ ("IwPQ") / IndexPreTransform ("IxPT") file or a
    CHIVFPQ1 image onto ``device``."""
    device = _default_device() if device is None else device
    if faiss_io.is_faiss_file(path):
        with open(path, "rb") as f:
            z = faiss_io.parse_index(f.read())
        if z["kind"] != "pretransform":
            return _ivfpq_from_dict(z, device)
        from .transform import IndexPreTransform, _linear_from_dict

        return IndexPreTransform([_linear_from_dict(t) for t in z["chain"]], _ivfpq_from_dict(z["index"], device))
    h = _lib.c_handle()
    L = _lib.load()
    _lib.check(L.ivfpq_load(str(path).encode(), device, ctypes.byref(h)))
    dims = [ctypes.c_int() for _ in range(5)]
    _lib.check(L.ivfpq_get_dims(h, *[ctypes.byref(v) for v in dims]))
    d, nlist, M, nbits, metric = [v.value for v in dims]
    idx = IndexIVFPQ(None, d, nlist, M, nbits, metric, device, _handle=h)
    if idx.is_trained:
        idx._sync_quantizer()
    return idx
