"""Hold-out reservation and training-set preparation.

Reference: ``Splitter`` (``core/.../stages/impl/tuning/Splitter.scala:58-182``; reserve 0.1, maxTrainingSample 1e6),
``DataSplitter`` (``DataSplitter.scala:73-98``: downsample to ``maxTrainingSample``), ``DataBalancer``
(``DataBalancer.scala:84-303``: up/down-sample the minority class to ``sampleFraction``) and ``DataCutter``
(``DataCutter.scala:78-334``: keep at most ``maxLabelCategories`` labels above ``minLabelFraction``).

Splitters work on row-index tensors (no data copies): sampling masks come from a seeded
counter-based RNG so every rank of a sharded dataset draws the same decision for a global row id.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from ..uid import make_uid


def _s64(c: int) -> int:
    """Reinterpret an unsigned 64-bit constant as the signed int64 torch arithmetic wraps with."""
    c &= (1 << 64) - 1
    return c - (1 << 64) if c >= (1 << 63) else c


_M63 = 0x7FFFFFFFFFFFFFFF


def _row_uniform_hip(row_ids: torch.Tensor, offs) -> torch.Tensor:
    """One fused HIP pass (ops/csrc/hip/boost_kernels.hip) for device row ids: ``[len(offs), n]``."""
    from ..ops import _native as N
    from ..ops.staging import to_device
    rid = row_ids.to(torch.int64).contiguous()
    out = torch.empty(len(offs), rid.shape[0], dtype=torch.float64, device=rid.device)
    o = to_device(list(offs), rid.device, np.int64)
    N.check(N.hip().tmog_hip_row_uniform(N.ptr(rid), rid.shape[0], N.ptr(o), len(offs), N.ptr(out),
                                         N.stream(rid.device)), "row_uniform")
    return out


def row_uniform(row_ids: torch.Tensor, seed: int, stream: int = 0) -> torch.Tensor:
    """Deterministic U[0,1) per global row id (splitmix64-style hash), identical on any device / shard."""
    off = _s64(int(seed) * 0x632BE59BD9B4E019 + stream * 0x2545F4914F6CDD1D)
    if row_ids.is_cuda and row_ids.numel():
        return _row_uniform_hip(row_ids, [off])[0]
    x = row_ids.to(torch.int64) * _s64(0x1E3779B97F4A7C15) + off
    x = x & _M63
    x = ((x ^ (x >> 30)) * _s64(0x2F58476D1CE4E5B9)) & _M63
    x = ((x ^ (x >> 27)) * _s64(0x14C3124B4B69A5C5)) & _M63
    x = x ^ (x >> 31)
    return (x >> 10).to(torch.float64) / float(1 << 53)


def row_uniform_multi(row_ids: torch.Tensor, seeds, stream: int = 0) -> torch.Tensor:
    """``row_uniform`` for several seeds at once: ``[len(seeds), n]`` (one fused pass, no per-seed launches)."""
    offs = [_s64(int(sd) * 0x632BE59BD9B4E019 + stream * 0x2545F4914F6CDD1D) for sd in seeds]
    if row_ids.is_cuda and row_ids.numel():
        return _row_uniform_hip(row_ids, offs)
    off = torch.tensor(offs, dtype=torch.int64, device=row_ids.device)[:, None]
    x = row_ids.to(torch.int64)[None, :] * _s64(0x1E3779B97F4A7C15) + off
    x = x & _M63
    x = ((x ^ (x >> 30)) * _s64(0x2F58476D1CE4E5B9)) & _M63
    x = ((x ^ (x >> 27)) * _s64(0x14C3124B4B69A5C5)) & _M63
    x = x ^ (x >> 31)
    return (x >> 10).to(torch.float64) / float(1 << 53)


class Splitter:
    reserve_test_fraction = 0.1

    def __init__(self, seed: Optional[int] = None, reserve_test_fraction: float = 0.1,
                 max_training_sample: int = 1_000_000, uid: Optional[str] = None):
        self.uid = uid or make_uid(type(self).__name__)
        self.seed = int(np.random.randint(0, 2 ** 31 - 1)) if seed is None else int(seed)
        self.reserve_test_fraction = reserve_test_fraction
        self.max_training_sample = max_training_sample
        self.down_sample_fraction = 1.0
        self.summary: Optional[Dict] = None

    def split(self, row_ids: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(train mask, test mask) of ``randomSplit([1 - f, f])``."""
        u = row_uniform(row_ids, self.seed, 1)
        test = u < self.reserve_test_fraction
        return ~test, test

    def pre_validation_prepare(self, y, n_total: Optional[int] = None) -> Dict:
        """Prepare from the labels: a tensor, or their value counts ``{label: count}`` (what every
        splitter needs -- data-parallel callers merge per-rank counts instead of gathering labels)."""
        raise NotImplementedError

    def validation_prepare(self, row_ids: torch.Tensor, y: torch.Tensor, stream: int = 7) -> torch.Tensor:
        """Boolean mask of rows kept for training."""
        self._check_prepared()
        return torch.ones(row_ids.shape[0], dtype=torch.bool, device=row_ids.device)

    def _check_prepared(self):
        """``Splitter.checkPreconditions`` (Splitter.scala:87)."""
        if self.summary is None:
            raise RuntimeError("requirement failed: Cannot call validationPrepare until preValidationPrepare has "
                               "been called")

    def params(self) -> Dict:
        return {"seed": self.seed, "reserveTestFraction": self.reserve_test_fraction,
                "maxTrainingSample": self.max_training_sample}

    def to_json(self):
        return {"className": type(self).__name__, "uid": self.uid, "params": self.params()}


def label_counts(y) -> Dict[float, int]:
    """``{label value: count}`` of a label tensor (a dict is returned as is)."""
    if isinstance(y, dict):
        return y
    vals, cnt = torch.unique(y.to(torch.float64), return_counts=True)
    return dict(zip(vals.tolist(), cnt.tolist()))


class DataSplitter(Splitter):
    def pre_validation_prepare(self, y, n_total=None):
        if n_total is not None:
            n = int(n_total)
        else:
            n = int(sum(y.values())) if isinstance(y, dict) else int(y.shape[0])
        self.down_sample_fraction = min(self.max_training_sample / max(n, 1), 1.0)
        self.summary = {"className": "com.salesforce.op.stages.impl.tuning.DataSplitterSummary",
                        "preSplitterDataCount": n, "downSamplingFraction": self.down_sample_fraction}
        return self.summary

    def validation_prepare(self, row_ids, y, stream=7):
        self._check_prepared()
        if self.down_sample_fraction >= 1.0:
            return torch.ones(row_ids.shape[0], dtype=torch.bool, device=row_ids.device)
        return row_uniform(row_ids, self.seed, stream) < self.down_sample_fraction


class DataBalancer(Splitter):
    """Rebalance a binary label: minority up-sampled (with replacement) and majority down-sampled so the
    minority fraction reaches ``sample_fraction`` and the total stays <= ``max_training_sample``."""

    def __init__(self, sample_fraction: float = 0.1, **kw):
        super().__init__(**kw)
        self.sample_fraction = sample_fraction
        self.up_fraction = 1.0
        self.already_balanced = False
        self.positive_is_small = True

    def pre_validation_prepare(self, y, n_total=None):
        cnt = label_counts(y)
        pos = float(sum(c for v, c in cnt.items() if v > 0.5))
        neg = float(sum(c for v, c in cnt.items() if not v > 0.5))
        small, big = (pos, neg) if pos < neg else (neg, pos)
        self.positive_is_small = pos < neg
        total = small + big
        f = self.sample_fraction
        mx = self.max_training_sample
        if small / max(total, 1) >= f:
            self.already_balanced = True
            self.down_sample_fraction = min(mx / max(total, 1), 1.0)
            self.up_fraction = 1.0
            reported_up = 0.0        # DataBalancer.scala:233-234 reports 0.0 when already balanced
        else:
            down, up = self.get_proportions(small, big, f, mx)
            self.up_fraction, self.down_sample_fraction = up, min(down, 1.0)
            reported_up = self.up_fraction
        self.summary = {"className": "com.salesforce.op.stages.impl.tuning.DataBalancerSummary",
                        "positiveLabels": int(pos), "negativeLabels": int(neg), "desiredFraction": f,
                        "upSamplingFraction": reported_up, "downSamplingFraction": self.down_sample_fraction}
        return self.summary

    @staticmethod
    def get_proportions(small: float, big: float, f: float, max_training_sample: int) -> Tuple[float, float]:
        """``getProportions`` (DataBalancer.scala:84-115) -> (down-sample fraction of the big class, up-sample
        multiplier of the small one): the largest multiplier in (100, 50, 10, 5, 4, 3, 2) that neither overshoots
        the desired fraction nor the training-size cap, or, when the small class alone exceeds its share of the
        cap, both classes sampled to the cap."""
        small, big, mx = float(small), float(big), float(max_training_sample)

        def fits(mult):
            return mult * small * (1 - f) < f * big and mx * f > small * mult
        if small < mx * f:
            up = next((float(m) for m in (100, 50, 10, 5, 4, 3, 2) if fits(m)), 1.0)
            return (small * up / f - small * up) / big, up
        return (1 - f) * mx / big, (mx * f) / small

    def validation_prepare(self, row_ids, y, stream=7):
        """Boolean keep-mask; up-sampling is expressed as integer weights via :meth:`weights`."""
        return self.weights(row_ids, y, stream) > 0

    def weights(self, row_ids, y, stream=7) -> torch.Tensor:
        self._check_prepared()
        u = row_uniform(row_ids, self.seed, stream)
        if self.already_balanced:
            return (u < self.down_sample_fraction).to(torch.int64)
        small_mask = (y > 0.5) if self.positive_is_small else (y <= 0.5)
        big_keep = (u < self.down_sample_fraction).to(torch.int64)
        lam = self.up_fraction
        u2 = row_uniform(row_ids, self.seed, stream + 101)
        # rebalance (DataBalancer.scala:287-291): up > 1 samples the minority with replacement
        # (Poisson(up) multiplicities), up == 1 keeps it as is, up < 1 samples without replacement
        if lam > 1.0:
            k = torch.zeros_like(u2, dtype=torch.int64)
            p = math.exp(-lam)
            cdf, pk = p, p
            for i in range(1, 64):
                k += (u2 >= cdf).to(torch.int64)
                pk = pk * lam / i
                cdf = cdf + pk
                if 1.0 - cdf < 1e-15:
                    break
        elif lam == 1.0:
            k = torch.ones_like(u2, dtype=torch.int64)
        else:
            k = (u2 < lam).to(torch.int64)
        return torch.where(small_mask, k, big_keep)

    def params(self):
        d = super().params()
        d["sampleFraction"] = self.sample_fraction
        return d


class DataCutter(Splitter):
    """Multiclass preparation (``DataCutter.scala:84-245``): keep the most frequent labels (count descending, then
    label; at most ``max_label_categories``, each with fraction >= ``min_label_fraction``), drop the others'
    rows, and down-sample to ``max_training_sample`` of the whole data. The summary records the kept labels in
    that order, the first ``max_names_for_dropped_labels`` dropped labels and the number of dropped label
    categories; labels estimated once are reused by later prepares."""

    def __init__(self, max_label_categories: int = 100, min_label_fraction: float = 0.0,
                 max_names_for_dropped_labels: int = 10, **kw):
        super().__init__(**kw)
        self.max_label_categories = max_label_categories
        self.min_label_fraction = min_label_fraction
        self.max_names_for_dropped_labels = max_names_for_dropped_labels
        self.labels_kept = None
        self.labels_dropped = None
        self.labels_dropped_total = 0

    def _estimate(self, cnt: Dict[float, int]):
        tot = float(sum(cnt.values()))
        order = sorted(cnt.items(), key=lambda vc: (-vc[1], vc[0]))
        kept = [v for v, c in order if c / tot >= self.min_label_fraction][:self.max_label_categories]
        if not kept:
            raise RuntimeError(f"DataCutter dropped all labels with param settings: minLabelFraction = "
                               f"{self.min_label_fraction}, maxLabelCategories = {self.max_label_categories}. \n"
                               f"Label counts were: {order}")
        ks = set(kept)
        dropped = [v for v, _ in order if v not in ks]
        self.labels_kept = kept
        self.labels_dropped = dropped[:self.max_names_for_dropped_labels]
        self.labels_dropped_total = len(order) - len(kept)

    def pre_validation_prepare(self, y, n_total=None):
        cnt = label_counts(y)
        if self.labels_kept is None:
            self._estimate(cnt)
        n = int(sum(cnt.values())) if n_total is None else int(n_total)
        self.down_sample_fraction = min(self.max_training_sample / max(n, 1), 1.0)
        self.summary = {"className": "com.salesforce.op.stages.impl.tuning.DataCutterSummary",
                        "preSplitterDataCount": n, "downSamplingFraction": self.down_sample_fraction,
                        "labelsKept": list(self.labels_kept), "labelsDropped": list(self.labels_dropped),
                        "labelsDroppedTotal": int(self.labels_dropped_total)}
        return self.summary

    def validation_prepare(self, row_ids, y, stream=7):
        self._check_prepared()
        keep = torch.isin(y.to(torch.float64), torch.as_tensor(self.labels_kept, dtype=torch.float64, device=y.device))
        if self.down_sample_fraction < 1.0:
            keep &= row_uniform(row_ids, self.seed, stream) < self.down_sample_fraction
        return keep

    def params(self):
        d = super().params()
        d.update(maxLabelCategories=self.max_label_categories, minLabelFraction=self.min_label_fraction)
        return d
