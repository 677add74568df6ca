"""Vector pre-transforms: Faiss ``LinearTransform`` / ``OPQMatrix`` and
``IndexPreTransform``.

The reference's billion-scale indexes are "OPQ16,IVF262144,PQ16"
(``Chameleon/Faiss_experiments/bench_gpu_1bn.py:10-17``): an OPQ rotation
trained with the PQ (``bench_gpu_1bn.py:480-495``) is applied to every base
and query vector before the IVF-PQ, and the FPGA extraction reads the matrix
back out of the index (``my_faiss_extract_scripts/extract_FPGA_required_data.py:
162-165``: ``index.chain.at(0)`` -> ``A`` reshaped ``(d, d)``).

* ``apply`` runs on the GPU (``ivfpq_linear_transform_device``, k_linear_transform:
  a t-ordered fused-multiply-add chain, the order ``oracle.linear_transform``
  restates; Faiss's sgemm leaves the order to BLAS, so parity with Faiss itself
  is unpinned).
* ``OPQMatrix.train`` restates Faiss 1.7.1 ``OPQMatrix::train`` (centre the
  training set, random orthonormal start, then ``niter`` rounds of: rotate, PQ
  k-means (``niter_pq_0`` then ``niter_pq`` iterations, hot-started), encode /
  decode, orthogonal Procrustes by SVD).  It runs on the host in numpy/float64
  like Faiss's LAPACK path; its random start and k-means seeding are not Faiss's
  (Faiss is not importable here), so trained matrices are not Faiss's either.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib, faiss_io


class _Chain(list):
    """IndexPreTransform.chain: a list with the SWIG vector's ``at``
    (extract_FPGA_required_data.py:164)."""

    def at(self, i):
        return self[i]


def downcast_VectorTransform(vt):
    return vt


def write_VectorTransform(vt, path):
    """faiss.write_VectorTransform (bench_gpu_1bn.py:507): one "LTra" record."""
    if not vt.is_trained:
        raise RuntimeError("write_VectorTransform: transform is not trained")
    with open(path, "wb") as f:
        f.write(faiss_io.serialize_linear(vt.A, vt.b, vt.d_in, vt.d_out, True))


def read_VectorTransform(path):
    """faiss.read_VectorTransform (bench_gpu_1bn.py:510) -> LinearTransform."""
    with open(path, "rb") as f:
        t = faiss_io.parse_vector_transform(f.read())
    return _linear_from_dict(t)


def _linear_from_dict(t):
    lt = LinearTransform(t["d_in"], t["d_out"], t["have_bias"])
    if t["is_trained"]:
        lt.set_matrix(t["A"], t["b"])
    return lt


class LinearTransform:
    """y = x A^T (+ b); A: [d_out][d_in] float32 (Faiss layout)."""

    def __init__(self, d_in=0, d_out=0, have_bias=False):
        self.d_in = int(d_in)
        self.d_out = int(d_out)
        self.have_bias = bool(have_bias)
        self.A = None
        self.b = None
        self.is_trained = False
        self._dev = {}

    def set_matrix(self, A, b=None):
        A = np.ascontiguousarray(A, np.float32).reshape(self.d_out, self.d_in)
        self.A = A
        self.b = None if b is None or not self.have_bias else np.ascontiguousarray(b, np.float32).reshape(self.d_out)
        self.is_trained = True
        self._dev = {}

    def _device_mats(self, device):
        import torch

        if device not in self._dev:
            AT = torch.from_numpy(np.ascontiguousarray(self.A.T)).to(f"cuda:{device}")
            b = torch.from_numpy(self.b).to(f"cuda:{device}") if self.b is not None else None
            self._dev[device] = (AT, b)
        return self._dev[device]

    def apply_device(self, x, stream=None):
        """x: torch float32 CUDA [n, d_in] -> y [n, d_out] on the same device (GPU kernel)."""
        import torch

        if not self.is_trained:
            raise RuntimeError("transform is not trained")
        if x.dim() != 2 or x.shape[1] != self.d_in or x.dtype != torch.float32 or not x.is_cuda:
            raise RuntimeError(f"apply_device: x must be a float32 CUDA tensor [n, {self.d_in}]")
        x = x.contiguous()
        AT, b = self._device_mats(x.device.index)
        cur = torch.cuda.current_stream(x.device)
        if stream is None or int(stream) == cur.cuda_stream:
            y = torch.empty((x.shape[0], self.d_out), dtype=torch.float32, device=x.device)
            s = cur.cuda_stream
        else:
            # a caller's stream: it waits for the current stream (x's producer, the
            # copies of AT and b), and y is allocated on it (the caching allocator
            # then never hands y's block to the current stream while it is in use);
            # x, AT and b are marked as used by it
            ext = torch.cuda.ExternalStream(int(stream), device=x.device)
            ext.wait_stream(cur)
            with torch.cuda.stream(ext):
                y = torch.empty((x.shape[0], self.d_out), dtype=torch.float32, device=x.device)
            for t in (x, AT, b):
                if t is not None:
                    t.record_stream(ext)
            s = int(stream)
        _lib.check(_lib.load().ivfpq_linear_transform_device(
            x.shape[0], self.d_in, self.d_out, AT.data_ptr(), b.data_ptr() if b is not None else None,
            x.data_ptr(), y.data_ptr(), ctypes.c_void_p(s)))
        return y

    def apply(self, x, device=0):
        """numpy [n, d_in] -> numpy [n, d_out], computed on GPU ``device``."""
        import torch

        x = torch.from_numpy(np.ascontiguousarray(x, np.float32)).to(f"cuda:{device}")
        y = self.apply_device(x)
        return y.cpu().numpy()

    apply_py = apply


class OPQMatrix(LinearTransform):
    """Faiss OPQMatrix(d, M, d2): an orthonormal rotation [d2][d] trained for M sub-quantizers."""

    def __init__(self, d=0, M=1, d2=-1):
        d2 = d if d2 == -1 else d2
        if d2 > d:
            raise RuntimeError("OPQMatrix: d_out > d_in is not supported")
        super().__init__(d, d2, False)
        self.M = int(M)
        self.niter = 50
        self.niter_pq = 4
        self.niter_pq_0 = 40
        self.max_train_points = 256 * 256
        self.seed = 1234
        if d2 % self.M:
            raise RuntimeError("OPQMatrix: d_out must be a multiple of M")

    @staticmethod
    def _pq_kmeans(xp, M, cb, niter, rng):
        n, d2 = xp.shape
        dsub = d2 // M
        for m in range(M):
            xs = xp[:, m * dsub:(m + 1) * dsub]
            if cb[m] is None:  # first round: 256 distinct training points
                cb[m] = xs[rng.choice(n, 256, replace=False)].copy()
            c = cb[m]
            for _ in range(niter):
                a = np.argmin((c * c).sum(1)[None, :] - 2.0 * xs @ c.T, axis=1)
                cnt = np.bincount(a, minlength=256)
                s = np.zeros_like(c)
                np.add.at(s, a, xs)
                nz = cnt > 0
                c[nz] = s[nz] / cnt[nz, None]  # empty centroids keep their position
        return cb

    @staticmethod
    def _pq_recons(xp, M, cb):
        n, d2 = xp.shape
        dsub = d2 // M
        out = np.empty_like(xp)
        for m in range(M):
            xs = xp[:, m * dsub:(m + 1) * dsub]
            c = cb[m]
            a = np.argmin((c * c).sum(1)[None, :] - 2.0 * xs @ c.T, axis=1)
            out[:, m * dsub:(m + 1) * dsub] = c[a]
        return out

    def train(self, x):
        x = np.ascontiguousarray(x, np.float32).reshape(-1, self.d_in)
        rng = np.random.default_rng(self.seed)
        if x.shape[0] > self.max_train_points:
            x = x[np.sort(rng.choice(x.shape[0], self.max_train_points, replace=False))]
        if x.shape[0] < 256:
            raise RuntimeError("OPQMatrix.train needs at least 256 training vectors")
        d, d2 = self.d_in, self.d_out
        xt = x.astype(np.float64)
        xt -= xt.mean(0, keepdims=True)
        if self.A is None:  # random orthonormal start, first d2 rows
            q, r = np.linalg.qr(rng.standard_normal((d, d)))
            A = (q * np.sign(np.diag(r))[None, :]).T[:d2].copy()
        else:
            A = self.A.astype(np.float64)
        cb = [None] * self.M
        for it in range(self.niter):
            xp = xt @ A.T
            cb = self._pq_kmeans(xp, self.M, cb, self.niter_pq_0 if it == 0 else self.niter_pq, rng)
            rec = self._pq_recons(xp, self.M, cb)
            u, _, vt = np.linalg.svd(xt.T @ rec, full_matrices=False)  # [d][d2] = U S V^T
            A = (u @ vt).T  # Procrustes: the rotation closest to mapping xt onto rec
        self.set_matrix(A.astype(np.float32))


class IndexPreTransform:
    """Faiss IndexPreTransform(chain, index): every vector is transformed on the GPU
    before the wrapped index sees it.  ``chain`` is a list of LinearTransform."""

    def __init__(self, chain, index):
        self.chain = _Chain(chain if isinstance(chain, (list, tuple)) else [chain])
        self.index = index
        self.d = self.chain[0].d_in
        self.metric_type = index.metric_type
        if self.chain[-1].d_out != index.d:
            raise RuntimeError("IndexPreTransform: the chain's output dimension differs from the index's")

    # Faiss attribute forwarding
    @property
    def ntotal(self):
        return self.index.ntotal

    @property
    def is_trained(self):
        return all(t.is_trained for t in self.chain) and self.index.is_trained

    @property
    def nprobe(self):
        return self.index.nprobe

    @nprobe.setter
    def nprobe(self, p):
        self.index.nprobe = p

    @property
    def device(self):
        return self.index.device

    def apply_chain(self, x):
        """numpy -> numpy through every transform (GPU)."""
        for t in self.chain:
            x = t.apply(x, self.index.device)
        return x

    def apply_chain_device(self, x, stream=None):
        for t in self.chain:
            x = t.apply_device(x, stream)
        return x

    def train(self, x):
        x = np.ascontiguousarray(x, np.float32).reshape(-1, self.d)
        for t in self.chain:
            if not t.is_trained:
                t.train(x)
            x = t.apply(x, self.index.device)
        if not self.index.is_trained:
            self.index.train(x)

    def add(self, x):
        self.index.add(self.apply_chain(np.ascontiguousarray(x, np.float32).reshape(-1, self.d)))

    def add_with_ids(self, x, ids):
        self.index.add_with_ids(self.apply_chain(np.ascontiguousarray(x, np.float32).reshape(-1, self.d)), ids)

    def search(self, x, k):
        import torch

        xd = torch.from_numpy(np.ascontiguousarray(x, np.float32).reshape(-1, self.d)).to(f"cuda:{self.index.device}")
        D, I = self.search_device(xd, k)
        return D.cpu().numpy(), I.cpu().numpy()

    def search_device(self, x, k, D=None, I=None, stream=None):
        return self.index.search_device(self.apply_chain_device(x, stream), k, D, I, stream)

    # the rest of the IVF-PQ surface callers reach through an OPQ index
    # (faiss_server.py / faiss_retriever.py: coarse step, preassigned search, wire requests)
    def coarse_device(self, x, Iq=None, Dq=None, stream=None):
        return self.index.coarse_device(self.apply_chain_device(x, stream), Iq, Dq, stream)

    def search_preassigned_device(self, x, k, Iq, Dq=None, D=None, I=None, stream=None):
        return self.index.search_preassigned_device(self.apply_chain_device(x, stream), k, Iq, Dq, D, I, stream)

    def search_preassigned(self, *args):
        """Both forms of IndexIVFPQ.search_preassigned, on the transformed queries."""
        if len(args) >= 7:
            n, x, k, Iq, Dq, D, I = args[:7]
            xt = self.apply_chain(np.ascontiguousarray(x, np.float32).reshape(-1, self.d))
            return self.index.search_preassigned(n, xt, k, Iq, Dq, D, I, *args[7:])
        x, k, Iq = args[:3]
        xt = self.apply_chain(np.ascontiguousarray(x, np.float32).reshape(-1, self.d))
        return self.index.search_preassigned(xt, k, Iq, *args[3:])

    def serve_request(self, msg, batch_size, dim, with_lists=False, nprobe=None, out=None):
        """A wire request on the pre-transform dimension: the queries are decoded,
        transformed on the GPU and re-encoded for the wrapped index."""
        from . import wire

        if dim != self.d:
            raise RuntimeError(f"dim={dim} does not match the index (d={self.d})")
        np_ = int(self.index.nprobe if nprobe is None else nprobe)
        if with_lists:
            k, q, lists = wire.decode_request_with_lists(msg, batch_size, dim, np_)
            msg2 = wire.encode_request_with_lists(self.apply_chain(np.array(q)), lists, batch_size, self.index.d,
                                                  np_, k)
        else:
            k, q = wire.decode_request(msg, batch_size, dim)
            msg2 = wire.encode_request(self.apply_chain(np.array(q)), k, batch_size, self.index.d)
        return self.index.serve_request(msg2, batch_size, self.index.d, with_lists=with_lists, nprobe=nprobe, out=out)

    def reset(self):
        self.index.reset()
