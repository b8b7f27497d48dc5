"""Geographic midpoint of Geolocation values (``aggregators/Geolocation.scala:43-138``,
``GeolocationAccuracy``, ``types/Geolocation.scala:121-190``).

A location becomes a Lucene spatial3d ``GeoPoint`` on the WGS84 ellipsoid (the unit-sphere direction of
(lat, lon) scaled to the ellipsoid surface) plus a box of half-width ``accuracy.rangeInUnits / 2`` around it.
The monoid is (coordinate sums, count, box minima, box maxima) -- columns 0-3 add, 4-6 take the minimum, 7-9
the maximum -- so partial results reduce as one sum, one min and one max on the device and over ranks. The
midpoint's latitude / longitude come from the summed direction; its accuracy is the finest one whose range
covers the widest side of the merged box (one location keeps its own accuracy). The reference builds the box's
upper z corner as z - d, not z + d; that is kept, since it decides the accuracy it reports.
"""
from __future__ import annotations

import math
from typing import List

import torch

EARTH_RADIUS_MILES = 3959.0
EQUATOR_MILES = 24901.0
# spatial3d PlanetModel.WGS84 axis scalings (equatorial / polar radius over the mean radius)
WGS84_XY = 6378137.0 / 6371008.7714
WGS84_Z = 6356752.314245 / 6371008.7714

# GeolocationAccuracy value -> rangeInMiles
ACCURACY_RANGE_MILES = {0: EQUATOR_MILES / 2, 1: 0.005, 2: 0.02, 3: 0.05, 4: 0.15, 5: 0.4, 6: 1.2, 7: 3.0, 8: 12.0,
                        9: 40.0, 10: 150.0}
_BY_RANGE = sorted(ACCURACY_RANGE_MILES.items(), key=lambda kv: kv[1])
STATS = 10


def accuracy_for_range_miles(miles: float) -> int:
    """``GeolocationAccuracy.forRangeInMiles``: the first accuracy (by range) whose range is at least 0.99 x
    ``miles``, else Unknown (0)."""
    for v, r in _BY_RANGE:
        if not r < miles * 0.99:
            return v
    return 0


def range_in_units(acc: torch.Tensor) -> torch.Tensor:
    lut = torch.tensor([ACCURACY_RANGE_MILES[k] for k in range(11)], dtype=torch.float64, device=acc.device)
    a = acc.round().long().clamp(0, 10)
    return lut[a] / EARTH_RADIUS_MILES


def prepare(geo: torch.Tensor) -> torch.Tensor:
    """``[n, 3]`` (lat, lon, accuracy) -> ``[n, 10]`` monoid rows."""
    g = geo.to(torch.float64)
    lat, lon = torch.deg2rad(g[:, 0]), torch.deg2rad(g[:, 1])
    ux, uy, uz = torch.cos(lat) * torch.cos(lon), torch.cos(lat) * torch.sin(lon), torch.sin(lat)
    mag = 1.0 / torch.sqrt((ux * ux + uy * uy) / (WGS84_XY * WGS84_XY) + uz * uz / (WGS84_Z * WGS84_Z))
    x, y, z = mag * ux, mag * uy, mag * uz
    d = range_in_units(g[:, 2]) / 2.0
    one = torch.ones_like(x)
    return torch.stack([x, y, z, one, x - d, y - d, z - d, x + d, y + d, z - d], 1)


def reduce_rows(P: torch.Tensor) -> torch.Tensor:
    """Fold ``[n, 10]`` monoid rows into one ``[10]`` (an empty input gives the zero: count 0)."""
    if P.shape[0] == 0:
        return torch.zeros(STATS, dtype=torch.float64, device=P.device)
    return torch.cat([P[:, :4].sum(0), P[:, 4:7].amin(0), P[:, 7:].amax(0)])


def reduce_by_key(P: torch.Tensor, slot: torch.Tensor, n_keys: int) -> torch.Tensor:
    """Segmented fold: rows with ``slot`` in [0, n_keys) -> ``[n_keys, 10]``."""
    out = torch.zeros(n_keys, STATS, dtype=torch.float64, device=P.device)
    out[:, 4:7] = float("inf")
    out[:, 7:] = -float("inf")
    if P.shape[0]:
        idx = slot.long()
        out[:, :4].index_add_(0, idx, P[:, :4])
        out[:, 4:7].scatter_reduce_(0, idx[:, None].expand(-1, 3), P[:, 4:7], reduce="amin", include_self=True)
        out[:, 7:].scatter_reduce_(0, idx[:, None].expand(-1, 3), P[:, 7:], reduce="amax", include_self=True)
    return out


def all_reduce(stats: torch.Tensor) -> torch.Tensor:
    """The monoid over data-parallel ranks: sums, minima and maxima in three collectives (no-op at world 1)."""
    from ..parallel import dp
    s = dp.sum_([stats[..., :4].contiguous()])[0]
    lo = dp.min_(stats[..., 4:7].contiguous())
    hi = dp.max_(stats[..., 7:].contiguous())
    return torch.cat([s, lo, hi], -1)


def present(stats) -> List[float]:
    """``GeolocationFunctions.present``: [lat, lon, accuracy] of a folded row, [] when it holds no location."""
    s = [float(v) for v in stats]
    if s[3] == 0.0:
        return []
    lat = math.degrees(math.atan2(s[2], math.sqrt(s[0] * s[0] + s[1] * s[1])))
    lon = math.degrees(math.atan2(s[1], s[0]))
    width = max(s[7] - s[4], s[8] - s[5], s[9] - s[6])
    return [lat, lon, float(accuracy_for_range_miles(width * EARTH_RADIUS_MILES))]
