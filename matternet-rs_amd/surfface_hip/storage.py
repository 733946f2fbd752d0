"""On-disk interchange with the reference ecosystem.

Mirror of the parquet layouts the reference writes for the path's outputs, so
a Laplacian / lambda vector produced here loads with the reference's own
readers and vice versa:
  * save_sparse_matrix / load_sparse_matrix  src_legacy/storage/parquet.rs:412-583
      COO triplets, schema (name_id Utf8, n_rows UInt64, n_cols UInt64,
      nnz UInt64, row UInt64, col UInt64, value Float64), all non-null,
      Snappy, file "<name_id>.parquet"; rows in CSR order.  Loading rebuilds
      the CSR like sprs TriMat::to_csr (columns sorted, duplicates summed).
  * save_lambda / load_lambda                 src_legacy/storage/parquet.rs:728-880
      schema (name_id Utf8, n_values UInt64, row_index UInt64, lambda Float64);
      an empty vector is an error (the reference's StorageError::Invalid).
Host-side I/O (pyarrow); device tensors are copied to the host first.
"""
from __future__ import annotations

import os

import numpy as np

try:
    import pyarrow as pa
    import pyarrow.parquet as pq
except ImportError as e:  # pragma: no cover - pyarrow ships in this image
    raise ImportError("surfface_hip.storage needs pyarrow") from e

SPARSE_SCHEMA = pa.schema([
    pa.field("name_id", pa.utf8(), nullable=False),
    pa.field("n_rows", pa.uint64(), nullable=False),
    pa.field("n_cols", pa.uint64(), nullable=False),
    pa.field("nnz", pa.uint64(), nullable=False),
    pa.field("row", pa.uint64(), nullable=False),
    pa.field("col", pa.uint64(), nullable=False),
    pa.field("value", pa.float64(), nullable=False),
])

LAMBDA_SCHEMA = pa.schema([
    pa.field("name_id", pa.utf8(), nullable=False),
    pa.field("n_values", pa.uint64(), nullable=False),
    pa.field("row_index", pa.uint64(), nullable=False),
    pa.field("lambda", pa.float64(), nullable=False),
])


def _host(a):
    return a.detach().cpu().numpy() if hasattr(a, "detach") else np.asarray(a)


def save_sparse_matrix(matrix, path: str, name_id: str) -> str:
    """matrix: CsrMatrix (device) or (indptr, indices, values, shape).  Writes
    <path>/<name_id>.parquet; returns the file path."""
    if isinstance(matrix, tuple):
        indptr, indices, values, shape = matrix
    else:
        indptr, indices, values, shape = matrix.indptr, matrix.indices, matrix.values, matrix.shape
    ip = _host(indptr).astype(np.int64)
    ix = _host(indices).astype(np.uint64)
    iv = _host(values).astype(np.float64)
    n_rows, n_cols = int(shape[0]), int(shape[1])
    nnz = int(ip[-1] - ip[0])
    rows = np.repeat(np.arange(n_rows, dtype=np.uint64), np.diff(ip))
    table = pa.Table.from_arrays([
        pa.array([name_id] * nnz, type=pa.utf8()),
        pa.array(np.full(nnz, n_rows, np.uint64)),
        pa.array(np.full(nnz, n_cols, np.uint64)),
        pa.array(np.full(nnz, nnz, np.uint64)),
        pa.array(rows),
        pa.array(ix[ip[0]:ip[-1]]),
        pa.array(iv[ip[0]:ip[-1]]),
    ], schema=SPARSE_SCHEMA)
    fp = os.path.join(path, f"{name_id}.parquet")
    pq.write_table(table, fp, compression="snappy")
    return fp


def load_sparse_matrix(path: str):
    """-> (indptr int64, indices int32, values f64, shape) like TriMat::to_csr
    (rows in order, columns sorted, duplicate triplets summed)."""
    t = pq.read_table(path)
    if t.num_rows == 0:
        raise ValueError("No data in parquet file")  # parquet.rs:581
    n_rows = int(t.column("n_rows")[0].as_py())
    n_cols = int(t.column("n_cols")[0].as_py())
    r = t.column("row").to_numpy().astype(np.int64)
    c = t.column("col").to_numpy().astype(np.int64)
    v = t.column("value").to_numpy().astype(np.float64)
    order = np.lexsort((c, r))
    r, c, v = r[order], c[order], v[order]
    if len(r):
        new = np.ones(len(r), bool)
        new[1:] = (r[1:] != r[:-1]) | (c[1:] != c[:-1])
        seg = np.cumsum(new) - 1
        v = np.bincount(seg, weights=v) if not np.all(new) else v
        r, c = r[new], c[new]
    indptr = np.zeros(n_rows + 1, np.int64)
    np.add.at(indptr, r + 1, 1)
    return np.cumsum(indptr), c.astype(np.int32), v, (n_rows, n_cols)


def save_lambda(lambdas, path: str, name_id: str) -> str:
    lam = _host(lambdas).astype(np.float64).ravel()
    n = len(lam)
    if n == 0:
        raise ValueError("Cannot save empty lambda vector")  # parquet.rs:737-741
    table = pa.Table.from_arrays([
        pa.array([name_id] * n, type=pa.utf8()),
        pa.array(np.full(n, n, np.uint64)),
        pa.array(np.arange(n, dtype=np.uint64)),
        pa.array(lam),
    ], schema=LAMBDA_SCHEMA)
    fp = os.path.join(path, f"{name_id}.parquet")
    pq.write_table(table, fp, compression="snappy")
    return fp


def load_lambda(path: str) -> np.ndarray:
    """The lambda column in file order (parquet.rs:826-867)."""
    return pq.read_table(path).column("lambda").to_numpy().astype(np.float64)
