"""faiss_amd — Faiss-compatible IVF-PQ search on AMD MI355X (gfx950).

Drop-in for the ``faiss`` calls Chameleon's callers make on its IVF-PQ path
(``import faiss_amd as faiss``); every search, train and add runs in the
hand-written HIP kernels of ``libivfpq.so`` through its C-ABI
(``include/ivfpq.h``).  The library is loaded on first use.
"""
from . import datasets  # noqa: F401  (pure numpy)
from .index import (  # noqa: F401
    MAX_K,
    METRIC_INNER_PRODUCT,
    METRIC_L2,
    IndexFlatIP,
    IndexFlatL2,
    IndexIVFPQ,
    ParameterSpace,
    downcast_index,
    extract_index_ivf,
    get_num_gpus,
    index_factory,
    merge_topk_device,
    overlap_built,
    read_index,
    swig_ptr,
    vector_to_array,
    write_index,
)
from .transform import (  # noqa: F401
    IndexPreTransform,
    LinearTransform,
    OPQMatrix,
    downcast_VectorTransform,
    read_VectorTransform,
    write_VectorTransform,
)
from . import contrib  # noqa: F401
from .contrib import ivf_tools  # noqa: F401

__version__ = "0.1.0"
