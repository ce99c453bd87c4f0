"""Synthetic test matrices of BASELINE.json (CSR, sorted, int32 columns).

Vectorised generators that scale to the 3-D 215^3 config (n = 9,938,375,
nnz = 69,291,275) without building a Kronecker product.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


def _stencil_csr(dims, diag, r0=0, r1=None, col_dtype=np.int32):
    """Rows [r0, r1) of the Dirichlet stencil matrix on grid ``dims`` (CSR,
    global column indices, sorted)."""
    dims = tuple(int(d) for d in dims)
    n_all = int(np.prod(dims))
    r1 = n_all if r1 is None else r1
    idx = np.arange(r0, r1, dtype=np.int64)
    n = len(idx)
    coords, stride, strides = [], 1, []
    for d in dims:  # first dimension is the fastest (column-major grid)
        coords.append((idx // stride) % d)
        strides.append(stride)
        stride *= d
    offsets = []  # increasing column offset: -s_last .. -s_0, 0, +s_0 .. +s_last
    for k in reversed(range(len(dims))):
        offsets.append((-strides[k], coords[k] > 0))
    offsets.append((0, None))
    for k in range(len(dims)):
        offsets.append((strides[k], coords[k] < dims[k] - 1))
    counts = np.ones(n, dtype=np.int64)
    for off, m in offsets:
        if m is not None:
            counts += m
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(counts, out=rowptr[1:])
    nnz = int(rowptr[-1])
    col = np.empty(nnz, dtype=col_dtype)
    val = np.empty(nnz, dtype=np.float64)
    pos = rowptr[:-1].copy()
    for off, m in offsets:
        if m is None:
            rows, p = idx, pos
            col[p] = rows
            val[p] = diag
            pos += 1
        else:
            rows = idx[m]
            p = pos[m]
            col[p] = rows + off
            val[p] = -1.0
            pos[m] += 1
    del coords, idx, pos
    return rowptr, col, val


WORKLOADS = {
    # name: (grid dims, diagonal)
    "lap2d": (2, 4.0),
    "lap3d": (3, 6.0),
}


def laplacian_2d(N: int) -> sp.csr_matrix:
    """5-point Dirichlet Laplacian on N x N (stencil 4, -1): BASELINE config 2."""
    rowptr, col, val = _stencil_csr((N, N), 4.0)
    return sp.csr_matrix((val, col, rowptr), shape=(N * N, N * N))


def laplacian_3d(N: int) -> sp.csr_matrix:
    """7-point Dirichlet Laplacian on N^3 (stencil 6, -1): BASELINE configs 3-4."""
    rowptr, col, val = _stencil_csr((N, N, N), 6.0)
    return sp.csr_matrix((val, col, rowptr), shape=(N ** 3, N ** 3))


def laplacian_rows(dim: int, N: int, r0: int, r1: int):
    """Rows [r0, r1) of the 2-D/3-D Laplacian with global int64 columns (a
    row slab of the distributed config 4): (rowptr, col, val)."""
    diag = 4.0 if dim == 2 else 6.0
    return _stencil_csr((N,) * dim, diag, r0, r1, col_dtype=np.int64)


def slab_bounds(n: int, nranks: int, plane: int = 1):
    """Contiguous row slabs aligned to whole planes (z-slabs for 3-D)."""
    nplanes = n // plane
    return [(plane * (nplanes * r // nranks)) for r in range(nranks)] + [n]


def diagonal(a) -> sp.csr_matrix:
    """``sparse(diag(a))`` -- BASELINE config 1 and the reference's diagonal tests."""
    a = np.asarray(a, dtype=np.float64)
    n = len(a)
    return sp.csr_matrix((a, np.arange(n, dtype=np.int32), np.arange(n + 1, dtype=np.int64)), shape=(n, n))


def circuit_like(n_side: int, seed: int = 0, keep: float = 0.8, long_frac: float = 0.3, span: int = 4
                 ) -> sp.csr_matrix:
    """Synthetic stand-in for SuiteSparse G3_circuit (BASELINE config 5; the
    .mtx is not in this container): the conductance matrix of a random
    resistor network, SPD and irregular.  An n_side^2 grid keeps each
    nearest-neighbour edge with probability ``keep``, adds ``long_frac * n``
    local long-range edges (offsets up to ``span`` grid rows), conductances
    U(0.1, 1), and grounds every node with U(1e-3, 1e-2).  At n_side = 1259
    (n = 1,585,081) it has ~4.8 nonzeros per row like G3_circuit (n =
    1,585,478, nnz = 7,660,826)."""
    N = int(n_side)
    n = N * N
    rng = np.random.default_rng(seed)
    idx = np.arange(n, dtype=np.int64).reshape(N, N)
    ei = np.concatenate([idx[:, :-1].ravel(), idx[:-1, :].ravel()])
    ej = np.concatenate([idx[:, 1:].ravel(), idx[1:, :].ravel()])
    m = rng.random(len(ei)) < keep
    ei, ej = ei[m], ej[m]
    nl = int(long_frac * n)
    li = rng.integers(0, n, nl)
    lj = li + rng.integers(1, span * N, nl)
    ok = lj < n
    ei = np.concatenate([ei, li[ok]])
    ej = np.concatenate([ej, lj[ok]])
    g = rng.uniform(0.1, 1.0, len(ei))
    deg = np.bincount(ei, g, n) + np.bincount(ej, g, n)
    ground = rng.uniform(1.0e-3, 1.0e-2, n)
    d = np.arange(n, dtype=np.int64)
    A = sp.csr_matrix((np.concatenate([-g, -g, deg + ground]),
                       (np.concatenate([ei, ej, d]), np.concatenate([ej, ei, d]))), shape=(n, n))
    A.sum_duplicates()
    A.sort_indices()
    A.indices = A.indices.astype(np.int32)
    return A


def _open_text(path: str):
    if path.endswith(".gz"):
        import gzip
        return gzip.open(path, "rt")
    return open(path)


def read_matrix_market(path: str) -> sp.csr_matrix:
    """Coordinate MatrixMarket reader (real/integer/pattern, general/symmetric;
    ``.mtx`` or ``.mtx.gz``).  The entries go through pandas' C parser
    (G3_circuit's 4.6M lines in a few seconds), or numpy.loadtxt without it."""
    with _open_text(path) as f:
        header = f.readline().lower().split()
        if len(header) < 5 or header[0] != "%%matrixmarket":
            raise ValueError("not a MatrixMarket file: %s" % path)
        if header[2] != "coordinate":
            raise ValueError("only coordinate MatrixMarket files are supported: %s" % path)
        field, symm = header[3], header[4]
        if field == "complex":
            raise ValueError("complex MatrixMarket matrices are not supported: %s" % path)
        line = f.readline()
        while line.startswith("%") or not line.strip():
            line = f.readline()
        m, n, nz = (int(t) for t in line.split()[:3])
        ncols = 2 if field == "pattern" else 3
        try:
            import pandas as pd
            data = pd.read_csv(f, sep=r"\s+", header=None, nrows=nz, usecols=range(ncols), comment="%",
                               dtype=np.float64, engine="c", float_precision="round_trip").to_numpy()
        except ImportError:  # pragma: no cover
            data = np.loadtxt(f, ndmin=2, max_rows=nz, usecols=range(ncols))
    if data.shape[0] != nz:
        raise ValueError("MatrixMarket %s: expected %d entries, read %d" % (path, nz, data.shape[0]))
    i = data[:, 0].astype(np.int64) - 1
    j = data[:, 1].astype(np.int64) - 1
    v = np.ones(len(i)) if field == "pattern" else data[:, 2].astype(np.float64)
    if symm in ("symmetric", "hermitian", "skew-symmetric"):
        off = i != j
        vt = -v[off] if symm == "skew-symmetric" else v[off]
        i, j, v = np.concatenate([i, j[off]]), np.concatenate([j, i[off]]), np.concatenate([v, vt])
    A = sp.csr_matrix((v, (i, j)), shape=(m, n))
    A.sum_duplicates()
    A.sort_indices()
    return A


def read_suitesparse_mat(path: str) -> sp.csr_matrix:
    """``load(path); A = Problem.A`` (test_restarted_ca_lanczos_all_matrices.m:
    25-26, test_restart_general_matrices.m:10-12): the SuiteSparse MATLAB
    format.  scipy.io.loadmat reads MAT v4/v5/v7 without executing anything
    from the file; v7.3 (HDF5) files need h5py, which this image lacks -- use
    the collection's MatrixMarket download for those."""
    import scipy.io
    try:
        d = scipy.io.loadmat(path, squeeze_me=True, struct_as_record=False)
    except NotImplementedError as e:  # MAT v7.3
        raise ValueError("%s is a MAT v7.3 (HDF5) file; h5py is not available -- use the .mtx form" % path) from e
    if "Problem" in d:
        A = getattr(d["Problem"], "A", None)
    else:
        A = d.get("A")
    if A is None or not sp.issparse(A):
        raise ValueError("%s holds no sparse Problem.A" % path)
    A = sp.csr_matrix(A, dtype=np.float64)
    A.sum_duplicates()
    A.sort_indices()
    return A


def load_matrix(path: str) -> sp.csr_matrix:
    """A matrix file of the reference's test suite as canonical CSR with int32
    columns: SuiteSparse ``.mat`` or MatrixMarket ``.mtx[.gz]``."""
    low = path.lower()
    if low.endswith(".mat"):
        A = read_suitesparse_mat(path)
    elif low.endswith(".mtx") or low.endswith(".mtx.gz") or low.endswith(".mm"):
        A = read_matrix_market(path)
    else:
        raise ValueError("unknown matrix file type: %s (expected .mat, .mtx or .mtx.gz)" % path)
    if A.shape[0] != A.shape[1]:
        raise ValueError("ERROR: Matrix %s is not square." % path)  # get_matrix_info.m:21
    A = to_csr(A)
    A.indices = A.indices.astype(np.int32)
    return A


def to_csr(A) -> sp.csr_matrix:
    """Canonical CSR (sorted, summed duplicates) with int32 column indices."""
    A = sp.csr_matrix(A)
    if not A.has_canonical_format:
        A = A.copy()
        A.sum_duplicates()
    A.sort_indices()
    return A
