"""Columnar storage for features (replaces Spark rows).

Every raw or derived feature is one column of a :class:`~transmogrifai_amd.data.dataset.Dataset`.
Storage is chosen by the feature type's ``kind``:

* ``numeric``  -> :class:`NumericColumn`: ``values`` tensor + ``valid`` bool mask (device resident)
* ``text``     -> :class:`TextColumn`: dictionary codes (``int32``, -1 = null) + host vocabulary
  (Arrow-style; string work runs once per distinct value, never per row)
* ``vector``   -> :class:`VectorColumn`: dense ``[N, d]`` tensor + :class:`OpVectorMetadata`
* ``prediction`` -> :class:`PredictionColumn`: prediction / raw / probability tensors
* ``geo``      -> :class:`GeoColumn`: ``[N, 3]`` tensor + mask
* ``list``/``set``/``map`` -> :class:`ObjectColumn`: host object array (ragged data)
"""
from __future__ import annotations

from typing import Any, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..features import types as T
from .vector_metadata import OpVectorMetadata


def _as_index(idx, device):
    if isinstance(idx, torch.Tensor):
        return idx.to(device=device, dtype=torch.long)
    return torch.as_tensor(np.asarray(idx, dtype=np.int64), device=device)


class Column:
    ftype: type = T.FeatureType

    def __len__(self) -> int:
        raise NotImplementedError

    @property
    def device(self):
        return torch.device("cpu")

    def take(self, idx) -> "Column":
        raise NotImplementedError

    def to(self, device) -> "Column":
        return self

    def row(self, i: int) -> Any:
        """Python value of row ``i`` (``None``/empty collection when missing)."""
        raise NotImplementedError

    def to_list(self) -> List[Any]:
        return [self.row(i) for i in range(len(self))]

    def null_mask(self) -> torch.Tensor:
        """Bool tensor, True where the value is empty."""
        return torch.tensor([_is_empty(self.row(i)) for i in range(len(self))], dtype=torch.bool)

    @staticmethod
    def concat(cols: Sequence["Column"]) -> "Column":
        return cols[0].__class__._concat(cols)


def _is_empty(v):
    if v is None:
        return True
    if isinstance(v, (list, tuple, set, frozenset, dict)):
        return len(v) == 0
    if isinstance(v, np.ndarray):
        return v.size == 0
    return False


# ------------------------------------------------------------------------------------------ numeric
class NumericColumn(Column):
    def __init__(self, ftype, values: torch.Tensor, valid: Optional[torch.Tensor] = None):
        self.ftype = ftype
        self.values = values
        if valid is None:
            valid = torch.ones(values.shape[0], dtype=torch.bool, device=values.device)
        self.valid = valid

    def __len__(self):
        return int(self.values.shape[0])

    @property
    def device(self):
        return self.values.device

    def take(self, idx):
        i = _as_index(idx, self.values.device)
        return NumericColumn(self.ftype, self.values[i], self.valid[i])

    def to(self, device):
        return NumericColumn(self.ftype, self.values.to(device), self.valid.to(device))

    def row(self, i):
        if not bool(self.valid[i]):
            return None
        v = self.values[i].item()
        if issubclass(self.ftype, T.Binary):
            return bool(v)
        if issubclass(self.ftype, T.Integral):
            return int(v)
        return float(v)

    def to_list(self):
        vals = self.values.detach().cpu().tolist()
        ok = self.valid.detach().cpu().tolist()
        if issubclass(self.ftype, T.Binary):
            return [bool(v) if k else None for v, k in zip(vals, ok)]
        if issubclass(self.ftype, T.Integral):
            return [int(v) if k else None for v, k in zip(vals, ok)]
        return [float(v) if k else None for v, k in zip(vals, ok)]

    def null_mask(self):
        return ~self.valid

    def as_double(self) -> torch.Tensor:
        """Values as float64 (0 where missing)."""
        v = self.values.to(torch.float64)
        return torch.where(self.valid, v, torch.zeros_like(v))

    @staticmethod
    def from_values(ftype, values: Sequence[Any], device="cpu", dtype=None):
        n = len(values)
        valid = np.ones(n, dtype=bool)
        if dtype is None:
            dtype = {"bool": np.bool_, "int64": np.int64}.get(ftype.dtype, np.float64)
        arr = np.zeros(n, dtype=dtype)
        for i, v in enumerate(values):
            if isinstance(v, T.FeatureType):
                v = v.value
            if v is None or (isinstance(v, float) and v != v):
                valid[i] = False
            else:
                arr[i] = v
        if not ftype.nullable and not valid.all():
            raise T.NonNullableEmptyException(f"{ftype.__name__} cannot contain empty values")
        return NumericColumn(ftype, torch.as_tensor(arr, device=device), torch.as_tensor(valid, device=device))

    @classmethod
    def _concat(cls, cols):
        return NumericColumn(cols[0].ftype, torch.cat([c.values for c in cols]),
                             torch.cat([c.valid for c in cols]))


# --------------------------------------------------------------------------------------------- text
class TextColumn(Column):
    """Dictionary-encoded strings: ``codes[i]`` indexes ``vocab`` (``-1`` = null)."""

    def __init__(self, ftype, codes: torch.Tensor, vocab: Sequence[str]):
        self.ftype = ftype
        self.codes = codes
        # row subsets and device moves share their parent's vocabulary list (never mutated): the batch text
        # results cached per vocabulary object (utils/text.py) then serve the training rows and the hold-out alike
        self.vocab = vocab if isinstance(vocab, list) else list(vocab)

    def __len__(self):
        return int(self.codes.shape[0])

    @property
    def device(self):
        return self.codes.device

    def take(self, idx):
        i = _as_index(idx, self.codes.device)
        return TextColumn(self.ftype, self.codes[i], self.vocab)

    def to(self, device):
        return TextColumn(self.ftype, self.codes.to(device), self.vocab)

    def row(self, i):
        c = int(self.codes[i])
        return None if c < 0 else self.vocab[c]

    def to_list(self):
        v = self.vocab
        return [None if c < 0 else v[c] for c in self.codes.detach().cpu().tolist()]

    def null_mask(self):
        return self.codes < 0

    def compact(self) -> "TextColumn":
        """Drop vocabulary entries that are not referenced."""
        cpu = self.codes.cpu().numpy()
        used = np.unique(cpu[cpu >= 0])
        remap = np.full(len(self.vocab) + 1, -1, dtype=np.int32)
        remap[used] = np.arange(len(used), dtype=np.int32)
        new = np.where(cpu >= 0, remap[np.maximum(cpu, 0)], -1).astype(np.int32)
        return TextColumn(self.ftype, torch.as_tensor(new, device=self.codes.device),
                          [self.vocab[u] for u in used])

    def map_vocab(self, fn, out_type=None) -> "TextColumn":
        """Apply a string function once per distinct value (``None`` result = null)."""
        mapped = [fn(s) for s in self.vocab]
        uniq = {}
        remap = np.full(len(mapped), -1, dtype=np.int32)
        for j, m in enumerate(mapped):
            if m is None:
                continue
            if m not in uniq:
                uniq[m] = len(uniq)
            remap[j] = uniq[m]
        remap_t = torch.as_tensor(np.append(remap, -1), device=self.codes.device)
        idx = torch.where(self.codes >= 0, self.codes.long(), torch.full_like(self.codes.long(), len(mapped)))
        return TextColumn(out_type or self.ftype, remap_t[idx].to(torch.int32), list(uniq.keys()))

    @staticmethod
    def from_values(ftype, values: Sequence[Any], device="cpu"):
        import pandas as pd
        vals = [None if (v is None or (isinstance(v, float) and v != v)) else
                (v.value if isinstance(v, T.FeatureType) else str(v)) for v in values]
        codes, uniques = pd.factorize(pd.Series(vals, dtype=object), use_na_sentinel=True)
        return TextColumn(ftype, torch.as_tensor(codes.astype(np.int32), device=device),
                          [str(u) for u in uniques])

    @classmethod
    def _concat(cls, cols):
        vocab = []
        index = {}
        parts = []
        for c in cols:
            remap = np.empty(len(c.vocab) + 1, dtype=np.int32)
            for j, s in enumerate(c.vocab):
                if s not in index:
                    index[s] = len(vocab)
                    vocab.append(s)
                remap[j] = index[s]
            remap[-1] = -1
            cc = c.codes.cpu().numpy()
            parts.append(remap[np.where(cc >= 0, cc, len(c.vocab))])
        dev = cols[0].codes.device
        return TextColumn(cols[0].ftype, torch.as_tensor(np.concatenate(parts), device=dev), vocab)


# ------------------------------------------------------------------------------------------- vector
class VectorColumn(Column):
    """Dense feature vectors ``[n, width]``.

    A vector column is either one dense tensor or a *blocked view*: an ordered list of
    ``(block [n, w_b], column index or None)`` parts whose concatenation is the logical matrix.
    ``VectorsCombiner`` concatenates its inputs' blocks and the SanityChecker keep-mask selects columns
    of them without copying the feature matrix; consumers that only need some rows
    (the model selector's training sample, chunked scoring) call :meth:`take_rows`, which gathers
    those rows of the selected columns straight from the blocks (HIP ``gather_rows_cols_kernel``).
    ``values`` materialises the whole matrix on demand for every other consumer."""
    ftype = T.OPVector

    def __init__(self, values: Optional[torch.Tensor] = None, metadata: Optional[OpVectorMetadata] = None,
                 blocks: Optional[Sequence[Tuple[torch.Tensor, Optional[torch.Tensor]]]] = None):
        self.metadata = metadata
        if blocks is None:
            assert values is not None and values.dim() == 2, None if values is None else values.shape
            self._values = values
            self._blocks = None
            self._n, self._w = int(values.shape[0]), int(values.shape[1])
            return
        parts = []
        for t, idx in blocks:
            assert t.dim() == 2
            w = int(t.shape[1]) if idx is None else int(idx.numel())
            if w > 0:
                parts.append((t, idx))
        if not parts:
            t0 = blocks[0][0] if blocks else torch.zeros(0, 0)
            parts = [(t0[:, :0], None)]
        if len({int(t.shape[0]) for t, _ in parts}) != 1:
            raise ValueError("vector blocks differ in row count")
        self._values = parts[0][0] if len(parts) == 1 and parts[0][1] is None else None
        self._blocks = None if self._values is not None else parts
        self._n = int(parts[0][0].shape[0])
        self._w = sum(int(t.shape[1]) if i is None else int(i.numel()) for t, i in parts)

    @property
    def values(self) -> torch.Tensor:
        if self._values is not None:
            return self._values
        return self.take_rows(None)

    @values.setter
    def values(self, v: torch.Tensor):
        assert v.dim() == 2
        self._values, self._blocks = v, None
        self._n, self._w = int(v.shape[0]), int(v.shape[1])

    @property
    def is_blocked(self) -> bool:
        return self._blocks is not None

    @property
    def blocks(self) -> List[Tuple[torch.Tensor, Optional[torch.Tensor]]]:
        return list(self._blocks) if self._blocks is not None else [(self._values, None)]

    @property
    def dtype(self):
        return self.blocks[0][0].dtype

    def __len__(self):
        return self._n

    @property
    def width(self) -> int:
        return self._w

    @property
    def device(self):
        return self.blocks[0][0].device

    def take_rows(self, idx) -> torch.Tensor:
        """Dense ``[len(idx), width]`` rows (all rows when ``idx`` is None) of the logical matrix."""
        if self._values is not None:
            return self._values if idx is None else self._values.index_select(
                0, _as_index(idx, self._values.device))
        from ..ops.vector import gather_rows_cols
        return gather_rows_cols(self._blocks, None if idx is None else _as_index(idx, self.device), self._n)

    def select_columns(self, idx, metadata: Optional[OpVectorMetadata] = None) -> "VectorColumn":
        """Columns ``idx`` of the logical matrix as a blocked view (no copy)."""
        dev = self.device
        idx = torch.as_tensor(idx, dtype=torch.long).cpu()
        parts, off = [], 0
        bounds = []
        for t, ci in self.blocks:
            w = int(t.shape[1]) if ci is None else int(ci.numel())
            bounds.append((off, off + w, t, ci))
            off += w
        if idx.numel() and (int(idx.min()) < 0 or int(idx.max()) >= off):
            raise IndexError("column index out of range of the vector")
        # consecutive output columns that fall in the same block become one part
        k = 0
        ids = idx.tolist()
        while k < len(ids):
            j = next(b for b in range(len(bounds)) if bounds[b][0] <= ids[k] < bounds[b][1])
            lo, hi, t, ci = bounds[j]
            m = k
            while m < len(ids) and lo <= ids[m] < hi:
                m += 1
            local = torch.as_tensor(ids[k:m], dtype=torch.long) - lo
            src = local if ci is None else ci.cpu()[local]
            whole = ci is None and src.numel() == t.shape[1] and bool((src == torch.arange(t.shape[1])).all())
            parts.append((t, None if whole else src.to(dev)))
            k = m
        if not parts:
            parts = [(self.blocks[0][0][:, :0], None)]
        return VectorColumn(metadata=metadata if metadata is not None else self.metadata, blocks=parts)

    def take(self, idx):
        return VectorColumn(self.take_rows(idx), self.metadata)

    def to(self, device):
        return VectorColumn(self.values.to(device), self.metadata)

    def row(self, i):
        return self.take_rows(torch.tensor([i]))[0].detach().cpu().numpy().astype(np.float64)

    def to_list(self):
        a = self.values.detach().cpu().numpy().astype(np.float64)
        return [a[i] for i in range(a.shape[0])]

    def null_mask(self):
        dev = self.device
        return torch.zeros(len(self), dtype=torch.bool, device=dev) if self.width > 0 \
            else torch.ones(len(self), dtype=torch.bool, device=dev)

    @staticmethod
    def from_values(values, device="cpu", metadata=None):
        vs = [np.asarray(v.value if isinstance(v, T.FeatureType) else v, dtype=np.float64) for v in values]
        d = max((v.size for v in vs), default=0)
        arr = np.zeros((len(vs), d))
        for i, v in enumerate(vs):
            arr[i, :v.size] = v
        return VectorColumn(torch.as_tensor(arr, device=device), metadata)

    @classmethod
    def _concat(cls, cols):
        return VectorColumn(torch.cat([c.values for c in cols]), cols[0].metadata)


# --------------------------------------------------------------------------------------- prediction
class PredictionColumn(Column):
    ftype = T.Prediction

    def __init__(self, prediction: torch.Tensor, raw: Optional[torch.Tensor] = None,
                 probability: Optional[torch.Tensor] = None):
        self.prediction = prediction
        n = prediction.shape[0]
        self.raw = raw if raw is not None else torch.zeros(n, 0, dtype=prediction.dtype, device=prediction.device)
        self.probability = probability if probability is not None else \
            torch.zeros(n, 0, dtype=prediction.dtype, device=prediction.device)

    def __len__(self):
        return int(self.prediction.shape[0])

    @property
    def device(self):
        return self.prediction.device

    def take(self, idx):
        i = _as_index(idx, self.prediction.device)
        return PredictionColumn(self.prediction[i], self.raw[i], self.probability[i])

    def to(self, device):
        return PredictionColumn(self.prediction.to(device), self.raw.to(device), self.probability.to(device))

    def row(self, i):
        return T.Prediction(prediction=float(self.prediction[i]),
                            raw_prediction=self.raw[i].tolist(), probability=self.probability[i].tolist()).value

    def to_list(self):
        p = self.prediction.detach().cpu().tolist()
        r = self.raw.detach().cpu().tolist()
        q = self.probability.detach().cpu().tolist()
        return [T.Prediction(prediction=p[i], raw_prediction=r[i], probability=q[i]).value for i in range(len(p))]

    def null_mask(self):
        return torch.zeros(len(self), dtype=torch.bool, device=self.prediction.device)

    def score(self) -> torch.Tensor:
        """Positive-class score for binary problems, else the prediction."""
        if self.probability.shape[1] == 2:
            return self.probability[:, 1]
        if self.probability.shape[1] == 1:
            return self.probability[:, 0]
        return self.prediction

    @staticmethod
    def from_values(values, device="cpu"):
        preds = [T.Prediction(v) if isinstance(v, dict) else v for v in values]
        p = torch.tensor([x.prediction for x in preds], dtype=torch.float64, device=device)
        k_raw = max((len(x.raw_prediction) for x in preds), default=0)
        k_prob = max((len(x.probability) for x in preds), default=0)
        raw = torch.tensor([x.raw_prediction or [0.0] * k_raw for x in preds], dtype=torch.float64,
                           device=device).reshape(len(preds), k_raw)
        prob = torch.tensor([x.probability or [0.0] * k_prob for x in preds], dtype=torch.float64,
                            device=device).reshape(len(preds), k_prob)
        return PredictionColumn(p, raw, prob)

    @classmethod
    def _concat(cls, cols):
        return PredictionColumn(torch.cat([c.prediction for c in cols]), torch.cat([c.raw for c in cols]),
                                torch.cat([c.probability for c in cols]))


# ---------------------------------------------------------------------------------------------- geo
class GeoColumn(Column):
    ftype = T.Geolocation

    def __init__(self, values: torch.Tensor, valid: torch.Tensor):
        self.values = values
        self.valid = valid

    def __len__(self):
        return int(self.values.shape[0])

    @property
    def device(self):
        return self.values.device

    def take(self, idx):
        i = _as_index(idx, self.values.device)
        return GeoColumn(self.values[i], self.valid[i])

    def to(self, device):
        return GeoColumn(self.values.to(device), self.valid.to(device))

    def row(self, i):
        return self.values[i].tolist() if bool(self.valid[i]) else []

    def null_mask(self):
        return ~self.valid

    @staticmethod
    def from_values(values, device="cpu"):
        n = len(values)
        arr = np.zeros((n, 3))
        ok = np.zeros(n, dtype=bool)
        for i, v in enumerate(values):
            v = v.value if isinstance(v, T.FeatureType) else v
            if v:
                arr[i] = T.Geolocation(v).value
                ok[i] = True
        return GeoColumn(torch.as_tensor(arr, device=device), torch.as_tensor(ok, device=device))

    @classmethod
    def _concat(cls, cols):
        return GeoColumn(torch.cat([c.values for c in cols]), torch.cat([c.valid for c in cols]))


# ------------------------------------------------------------------------------------------- object
class ObjectColumn(Column):
    """Host-resident ragged values: lists, sets, maps."""

    def __init__(self, ftype, values: np.ndarray):
        self.ftype = ftype
        if not isinstance(values, np.ndarray) or values.dtype != object:
            arr = np.empty(len(values), dtype=object)
            for i, v in enumerate(values):
                arr[i] = v
            values = arr
        self.values = values

    def __len__(self):
        return len(self.values)

    def take(self, idx):
        if isinstance(idx, torch.Tensor):
            idx = idx.cpu().numpy()
        return ObjectColumn(self.ftype, self.values[np.asarray(idx, dtype=np.int64)])

    def row(self, i):
        return self.values[i]

    def to_list(self):
        return list(self.values)

    def null_mask(self):
        return torch.as_tensor(np.array([_is_empty(v) for v in self.values], dtype=bool))

    @staticmethod
    def from_values(ftype, values, device="cpu"):
        out = np.empty(len(values), dtype=object)
        for i, v in enumerate(values):
            out[i] = ftype(v.value if isinstance(v, T.FeatureType) else v).value
        return ObjectColumn(ftype, out)

    @classmethod
    def _concat(cls, cols):
        return ObjectColumn(cols[0].ftype, np.concatenate([c.values for c in cols]))


def column_from_values(ftype, values: Sequence[Any], device="cpu") -> Column:
    """Build the right column class for ``ftype`` from python values."""
    kind = ftype.kind
    if kind == "numeric":
        return NumericColumn.from_values(ftype, values, device)
    if kind == "text":
        return TextColumn.from_values(ftype, values, device)
    if kind == "vector":
        return VectorColumn.from_values(values, device)
    if kind == "prediction":
        return PredictionColumn.from_values(values, device)
    if kind == "geo":
        return GeoColumn.from_values(values, device)
    return ObjectColumn.from_values(ftype, values, device)
