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
  * save_dense_matrix / load_dense_matrix     src_legacy/storage/parquet.rs:215-400
      schema (name_id Utf8, n_rows UInt64, n_cols UInt64, col_0 .. col_{c-1}
      Float64), one row per matrix row, all non-null, Snappy; loading reads
      n_rows / n_cols from the first batch and checks the row count.
  * ArrowSpaceMetadata, save_metadata / load_metadata
                                              src_legacy/storage/parquet.rs:27-165
      "<name_id>_metadata.json" (serde_json pretty print of the struct:
      name_id, timestamp, n_rows, n_cols, builder_config {key: ConfigValue},
      files {key: FileInfo}); ConfigValue in serde's externally tagged form,
      e.g. {"F64": 0.1}, {"TauMode": "Median"}, {"OptionUsize": null}
      (surfface-pipeline/src/builder.rs:1533-1544).  The save_* functions
      write it when a builder_config is given (parquet.rs:312-330, 484-500).
Host-side I/O (pyarrow); device tensors are copied to the host first.
"""
from __future__ import annotations

import datetime
import json
import math
import os
from dataclasses import dataclass, field
from typing import Dict, Optional

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


class StorageError(ValueError):
    """The reference's StorageError::Invalid / Io (parquet.rs): bad or missing
    data in a file this module reads."""


# ConfigValue variants (builder.rs:1533-1544): serde's externally tagged form
CONFIG_VALUE_KINDS = ("Bool", "Usize", "F64", "U64", "String", "OptionF64", "OptionUsize",
                      "OptionU64", "TauMode", "OptionSamplerType")


def config_value(kind: str, value) -> dict:
    """ConfigValue::<kind>(value) as serde_json writes it: {"F64": 0.5},
    {"TauMode": "Median"} / {"TauMode": {"Fixed": 0.3}}, {"OptionUsize": null}."""
    if kind not in CONFIG_VALUE_KINDS:
        raise StorageError(f"unknown ConfigValue variant {kind!r}")
    return {kind: value}


@dataclass
class FileInfo:
    """parquet.rs:49-57."""
    filename: str
    file_type: str  # "dense" or "sparse"
    rows: int
    cols: int
    nnz: Optional[int] = None
    size_bytes: Optional[int] = None


def _finite_or_null(v):
    """serde_json's f64 serialisation: NaN and +-inf become null."""
    if isinstance(v, float) and not math.isfinite(v):
        return None
    if isinstance(v, dict):
        return {k: _finite_or_null(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [_finite_or_null(x) for x in v]
    return v


@dataclass
class ArrowSpaceMetadata:
    """parquet.rs:31-47 (field order as serialised)."""
    name_id: str
    timestamp: str = field(default_factory=lambda: datetime.datetime.now(
        datetime.timezone.utc).isoformat())
    n_rows: int = 0
    n_cols: int = 0
    builder_config: Dict[str, dict] = field(default_factory=dict)
    files: Dict[str, FileInfo] = field(default_factory=dict)

    def with_builder_config(self, config: Dict[str, dict]) -> "ArrowSpaceMetadata":
        self.builder_config = dict(config)
        return self

    def with_dimensions(self, rows: int, cols: int) -> "ArrowSpaceMetadata":
        self.n_rows, self.n_cols = int(rows), int(cols)
        return self

    def add_file(self, key: str, info: FileInfo) -> "ArrowSpaceMetadata":
        self.files[key] = info
        return self

    def get_config(self, key: str):
        return self.builder_config.get(key)

    def _typed(self, key, kinds):
        v = self.get_config(key)
        if v is None:
            return None
        (kind, val), = v.items()
        if kind not in kinds:
            # the reference's as_* accessors panic on a different variant
            raise StorageError(f"config {key!r} is {kind}, not {kinds[0]}")
        return val

    def lambda_eps(self) -> Optional[float]:
        """ConfigValue::as_f64 (surfface-pipeline/src/builder.rs:1569-1582):
        NaN reads as -1.0; another variant panics."""
        v = self._typed("lambda_eps", ("F64", "OptionF64"))
        if v is not None and isinstance(v, float) and math.isnan(v):
            return -1.0
        return v

    def lambda_k(self) -> Optional[int]:
        return self._typed("lambda_k", ("Usize", "OptionUsize"))

    def synthesis(self):
        """ConfigValue::as_tau_mode (builder.rs:1599-1604): None for any other
        variant (it does not panic, unlike as_f64 / as_usize)."""
        v = self.get_config("synthesis")
        if v is None:
            return None
        (kind, val), = v.items()
        return val if kind == "TauMode" else None

    def to_json(self) -> str:
        d = {"name_id": self.name_id, "timestamp": self.timestamp, "n_rows": self.n_rows,
             "n_cols": self.n_cols, "builder_config": self.builder_config,
             "files": {k: {"filename": f.filename, "file_type": f.file_type, "rows": f.rows,
                           "cols": f.cols, "nnz": f.nnz, "size_bytes": f.size_bytes}
                       for k, f in self.files.items()}}
        # serde_json::to_string_pretty: 2 spaces; a non-finite f64 is written
        # as null (serde_json never emits the bare NaN / Infinity tokens)
        return json.dumps(_finite_or_null(d), indent=2, allow_nan=False)

    @classmethod
    def from_json(cls, text: str) -> "ArrowSpaceMetadata":
        try:
            d = json.loads(text)
            files = {k: FileInfo(v["filename"], v["file_type"], int(v["rows"]), int(v["cols"]),
                                 v.get("nnz"), v.get("size_bytes"))
                     for k, v in d["files"].items()}
            for key, v in d["builder_config"].items():
                if not (isinstance(v, dict) and len(v) == 1 and next(iter(v)) in CONFIG_VALUE_KINDS):
                    raise ValueError(f"builder_config[{key!r}] is not a ConfigValue")
                # serde_json refuses null for a plain f64 (only the Option
                # variants take it): a non-finite F64 written as null does not
                # load back in the reference either (parity unpinned: no
                # reference fixture holds this case)
                (kind, val), = v.items()
                if kind in ("F64", "Usize", "U64", "Bool", "String") and val is None:
                    raise ValueError(f"builder_config[{key!r}]: null is not a valid {kind}")
            return cls(d["name_id"], d["timestamp"], int(d["n_rows"]), int(d["n_cols"]),
                       d["builder_config"], files)
        except (KeyError, TypeError, ValueError) as e:
            raise StorageError(f"Failed to parse metadata: {e}") from e


def save_metadata(metadata: ArrowSpaceMetadata, path: str, name_id: str) -> str:
    """parquet.rs:131-146: <path>/<name_id>_metadata.json."""
    fp = os.path.join(path, f"{name_id}_metadata.json")
    with open(fp, "w") as f:
        f.write(metadata.to_json())
    return fp


def load_metadata(path: str, name_id: str) -> ArrowSpaceMetadata:
    """parquet.rs:148-165."""
    fp = os.path.join(path, f"{name_id}_metadata.json")
    try:
        text = open(fp).read()
    except OSError as e:
        raise StorageError(f"Failed to read metadata: {e}") from e
    return ArrowSpaceMetadata.from_json(text)


def _write_metadata(path, name_id, fp, kind, n_rows, n_cols, nnz, builder_config):
    if builder_config is None:
        return
    info = FileInfo(f"{name_id}.parquet", kind, int(n_rows), int(n_cols), nnz,
                    os.path.getsize(fp) if os.path.exists(fp) else None)
    md = (ArrowSpaceMetadata(name_id).with_builder_config(builder_config)
          .with_dimensions(n_rows, n_cols).add_file("matrix", info))
    save_metadata(md, path, name_id)


def save_dense_matrix(matrix, path: str, name_id: str,
                      builder_config: Optional[Dict[str, dict]] = None) -> str:
    """parquet.rs:233-331: matrix [n_rows][n_cols] (tensor or array, stored
    as f64) -> <path>/<name_id>.parquet (+ the metadata JSON when a
    builder_config is given); returns the parquet path."""
    m = _host(matrix).astype(np.float64)
    if m.ndim != 2:
        raise StorageError("save_dense_matrix: a 2-D matrix is required")
    n_rows, n_cols = m.shape
    fields = [pa.field("name_id", pa.utf8(), nullable=False),
              pa.field("n_rows", pa.uint64(), nullable=False),
              pa.field("n_cols", pa.uint64(), nullable=False)]
    fields += [pa.field(f"col_{i}", pa.float64(), nullable=False) for i in range(n_cols)]
    arrays = [pa.array([name_id] * n_rows, type=pa.utf8()),
              pa.array(np.full(n_rows, n_rows, np.uint64)),
              pa.array(np.full(n_rows, n_cols, np.uint64))]
    arrays += [pa.array(np.ascontiguousarray(m[:, i])) for i in range(n_cols)]
    table = pa.Table.from_arrays(arrays, schema=pa.schema(fields))
    fp = os.path.join(path, f"{name_id}.parquet")
    pq.write_table(table, fp, compression="snappy")
    _write_metadata(path, name_id, fp, "dense", n_rows, n_cols, None, builder_config)
    return fp


def load_dense_matrix(path: str) -> np.ndarray:
    """parquet.rs:345-400 -> [n_rows][n_cols] f64 (the same matrix the
    reference rebuilds column-major)."""
    pf = pq.ParquetFile(path)
    n_rows = n_cols = None
    out = None
    off = 0
    for batch in pf.iter_batches():
        names = batch.schema.names
        if n_rows is None:
            if "n_rows" not in names:
                raise StorageError("n_rows column missing")
            if "n_cols" not in names:
                raise StorageError("n_cols column missing")
            n_rows = int(batch.column(names.index("n_rows"))[0].as_py())
            n_cols = int(batch.column(names.index("n_cols"))[0].as_py())
            out = np.zeros((n_rows, n_cols), np.float64)
        b = batch.num_rows
        if off + b > n_rows:
            raise StorageError(f"Parquet file contained more than {n_rows} rows")
        for c in range(n_cols):
            name = f"col_{c}"
            if name not in names:
                raise StorageError(f"Column {name} missing")
            out[off:off + b, c] = batch.column(names.index(name)).to_numpy()
        off += b
    if n_rows is None:
        raise StorageError("No data in parquet file")
    if off != n_rows:
        raise StorageError(f"Parquet file contained {off} rows, but metadata claimed {n_rows}")
    return out


def save_sparse_matrix(matrix, path: str, name_id: str,
                       builder_config: Optional[Dict[str, dict]] = None) -> str:
    """matrix: CsrMatrix (device) or (indptr, indices, values, shape).  Writes
    <path>/<name_id>.parquet (+ the metadata JSON when a builder_config is
    given, parquet.rs:484-500); returns the file path."""
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
    _write_metadata(path, name_id, fp, "sparse", n_rows, n_cols, nnz, builder_config)
    return fp


def load_sparse_matrix(path: str):
    """-> (indptr int64, indices int32, values f64, shape) like TriMat::to_csr
    (rows in order, columns sorted, duplicate triplets summed)."""
    t = pq.read_table(path)
    if t.num_rows == 0:
        raise StorageError("No data in parquet file")  # parquet.rs:581
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
        raise StorageError("Cannot save empty lambda vector")  # parquet.rs:737-741
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
