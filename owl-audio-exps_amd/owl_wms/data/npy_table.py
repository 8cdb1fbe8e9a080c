"""On-disk latent table (reference: owl_wms/data/npy_table.py:7-92).

Format, identical to the reference so tables written by either side load in the other:

* ``schema.json``   ``{"columns": [...], "array_columns": [...]}`` (written once, checked after);
* ``manifest.json`` one JSON object per row; an array column holds the file name
  ``{col}_{row}.npy``, every other column holds the value itself;
* ``{col}_{row}.npy`` ``np.save`` output (no pickle), read back memory-mapped.

Rows are memory-mapped rather than loaded: a 1536-frame dit_v4 window is 25 MB of fp32 latents
per row slice, and a loader worker only touches the frames it packs.
"""
import json
from pathlib import Path
from typing import Any, Iterable, List, Optional

import numpy as np

DEFAULT_COLUMNS = ["video", "audio", "mouse", "buttons", "tarball", "pt_idx", "missing", "truncated",
                   "seq_len"]
DEFAULT_ARRAY_COLUMNS = ["video", "audio", "mouse", "buttons"]


class NpyTable:
    default_columns = DEFAULT_COLUMNS
    default_array_columns = set(DEFAULT_ARRAY_COLUMNS)

    def __init__(self, directory: str, columns: Optional[List[str]] = None,
                 array_columns: Optional[Iterable[str]] = None):
        self.directory = Path(directory)
        self.directory.mkdir(parents=True, exist_ok=True)
        self.schema_path = self.directory / "schema.json"
        self.manifest_path = self.directory / "manifest.json"

        if self.schema_path.exists():
            schema = json.loads(self.schema_path.read_text())
            # npy_table.py:22-27: a reopened table must agree with what the caller asks for
            if columns is not None and list(columns) != schema["columns"]:
                raise AssertionError("columns mismatch")
            if array_columns is not None and set(array_columns) != set(schema["array_columns"]):
                raise AssertionError("array_columns mismatch")
            columns, array_columns = schema["columns"], schema["array_columns"]
        else:
            columns = list(columns or DEFAULT_COLUMNS)
            array_columns = list(array_columns or DEFAULT_ARRAY_COLUMNS)
            self.schema_path.write_text(json.dumps({"columns": columns, "array_columns": array_columns}))
        self.columns = list(columns)
        self.array_columns = set(array_columns)
        self.manifest = json.loads(self.manifest_path.read_text()) if self.manifest_path.exists() else []
        self._mmaps = {}

    def __len__(self):
        return len(self.manifest)

    def append(self, **row: Any) -> int:
        """npy_table.py:49-68: exactly the schema's columns; arrays to ``{col}_{idx}.npy``."""
        if set(row) != set(self.columns):
            raise ValueError(f"Expected columns {self.columns}, got {list(row)}")
        idx = len(self.manifest)
        entry = {}
        for col, val in row.items():
            if col in self.array_columns:
                name = f"{col}_{idx}.npy"
                with open(self.directory / name, "wb", buffering=8 << 20) as f:
                    np.save(f, np.ascontiguousarray(val), allow_pickle=False)
                entry[col] = name
            else:
                entry[col] = val
        self.manifest.append(entry)
        self.manifest_path.write_text(json.dumps(self.manifest))
        return idx

    def array(self, col: str, row: int) -> np.ndarray:
        """Memory-mapped array of one cell (cached per process; never pickled)."""
        key = (col, row)
        a = self._mmaps.get(key)
        if a is None:
            a = np.load(self.directory / self.manifest[row][col], mmap_mode="r", allow_pickle=False)
            self._mmaps[key] = a
        return a

    def get(self, columns: List[str], rows: Optional[Iterable[int]] = None) -> List[List[Any]]:
        """npy_table.py:79-92: column-major ``[[cell for row] for col]``."""
        unknown = set(columns) - set(self.columns)
        if unknown:
            raise KeyError(f"Unknown columns requested: {unknown}")
        rows = range(len(self.manifest)) if rows is None else list(rows)
        return [[self.array(c, r) if c in self.array_columns else self.manifest[r][c] for r in rows]
                for c in columns]

    def __getitem__(self, key):
        if isinstance(key, str):
            return self.get([key])[0]
        if isinstance(key, (list, tuple)):
            return self.get(list(key))
        raise KeyError(f"Invalid key: {key!r}")

    def __getstate__(self):
        # DataLoader workers re-open their own memory maps
        d = dict(self.__dict__)
        d["_mmaps"] = {}
        return d
