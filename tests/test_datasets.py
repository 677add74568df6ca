import numpy as np

from faiss_amd import datasets


def test_fvecs_ivecs_roundtrip(tmp_path):
    x = np.random.default_rng(0).standard_normal((7, 5)).astype(np.float32)
    datasets.fvecs_write(tmp_path / "a.fvecs", x)
    np.testing.assert_array_equal(datasets.fvecs_read(tmp_path / "a.fvecs"), x)
    g = np.arange(12, dtype=np.int32).reshape(3, 4)
    datasets.ivecs_write(tmp_path / "g.ivecs", g)
    np.testing.assert_array_equal(datasets.ivecs_read(tmp_path / "g.ivecs"), g)


def test_fbin_ibin(tmp_path):
    x = np.arange(12, dtype=np.float32).reshape(3, 4)
    with open(tmp_path / "x.fbin", "wb") as f:
        np.array([3, 4], np.int32).tofile(f)
        x.tofile(f)
    np.testing.assert_array_equal(np.asarray(datasets.mmap_fbin(tmp_path / "x.fbin")), x)
    with open(tmp_path / "g.ibin", "wb") as f:
        np.array([3, 4], np.int32).tofile(f)
        x.astype(np.int32).tofile(f)
    np.testing.assert_array_equal(datasets.read_ibin(tmp_path / "g.ibin"), x.astype(np.int32))


def test_recall_definitions():
    # R1@k (bench_polysemous_1bn.py:432-434) and R@k (bench_cpu_performance_OSDI.py:355-359)
    I = np.array([[1, 2, 3], [4, 5, 6]])
    gt = np.array([[2, 9, 9], [7, 4, 5]])
    r = datasets.recall_1_at(I, gt, (1, 2, 3))
    assert r == {1: 0.0, 2: 0.5, 3: 0.5}
    assert datasets.recall_at_k(I, gt, 3) == (1 + 2) / 6


def test_synthetic_generator_shape_and_determinism():
    a = datasets.synthetic_sift_like(1000, 32, seed=5, n_centres=10)
    b = datasets.synthetic_sift_like(1000, 32, seed=5, n_centres=10)
    np.testing.assert_array_equal(a, b)
    assert a.dtype == np.float32 and a.min() >= 0 and a.max() <= 255
    assert np.all(a == np.rint(a))


def test_brute_force_gt():
    rng = np.random.default_rng(1)
    xb = rng.integers(0, 10, (200, 8)).astype(np.float32)
    xq = rng.integers(0, 10, (5, 8)).astype(np.float32)
    gt = datasets.brute_force_gt(xb, xq, 4)
    dd = ((xq[:, None] - xb[None]) ** 2).sum(-1)
    for q in range(5):
        np.testing.assert_array_equal(gt[q], np.lexsort((np.arange(200), dd[q]))[:4])
