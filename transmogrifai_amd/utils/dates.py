"""Vectorized UTC calendar arithmetic on int64 epoch-millisecond tensors (no Joda/JVM).

``TimePeriod`` semantics of the reference (``features/.../stages/impl/feature/TimePeriod.scala``):
DayOfMonth [1,31], DayOfWeek [1,7] (Monday = 1), DayOfYear [1,366], HourOfDay [0,24),
MonthOfYear [1,12], WeekOfMonth [1,6], WeekOfYear [1,53] with ``WeekFields.of(MONDAY, 1)``.
Civil dates use Howard Hinnant's days-from-civil inverse, which runs unchanged on the GPU.
"""
from __future__ import annotations

import time

import torch

MS_PER_DAY = 86400000
TIME_PERIODS = {"DayOfMonth": (1, 31), "DayOfWeek": (1, 7), "DayOfYear": (1, 366), "HourOfDay": (0, 24),
                "MonthOfYear": (1, 12), "WeekOfMonth": (1, 6), "WeekOfYear": (1, 53)}
_CUM = torch.tensor([0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334], dtype=torch.int64)


def now_ms() -> int:
    return int(time.time() * 1000)


def _fdiv(a, b):
    return torch.div(a, b, rounding_mode="floor")


def civil(days: torch.Tensor):
    """days since epoch -> (year, month [1,12], day [1,31])."""
    z = days + 719468
    era = _fdiv(z, 146097)
    doe = z - era * 146097
    yoe = _fdiv(doe - _fdiv(doe, 1460) + _fdiv(doe, 36524) - _fdiv(doe, 146096), 365)
    y = yoe + era * 400
    doy = doe - (365 * yoe + _fdiv(yoe, 4) - _fdiv(yoe, 100))
    mp = _fdiv(5 * doy + 2, 153)
    d = doy - _fdiv(153 * mp + 2, 5) + 1
    m = torch.where(mp < 10, mp + 3, mp - 9)
    y = y + (m <= 2).to(y.dtype)
    return y, m, d


def _leap(y):
    return ((y % 4 == 0) & (y % 100 != 0)) | (y % 400 == 0)


def day_of_week(days):
    return (days + 3) % 7 + 1   # 1970-01-01 is a Thursday (ISO 4)


def fields(ms: torch.Tensor, period: str) -> torch.Tensor:
    ms = ms.to(torch.int64)
    days = _fdiv(ms, MS_PER_DAY)
    if period == "HourOfDay":
        return _fdiv(ms - days * MS_PER_DAY, 3600000)
    if period == "DayOfWeek":
        return day_of_week(days)
    y, m, d = civil(days)
    if period == "DayOfMonth":
        return d
    if period == "MonthOfYear":
        return m
    cum = _CUM.to(ms.device)
    doy = cum[m - 1] + d + (_leap(y) & (m > 2)).to(torch.int64)
    if period == "DayOfYear":
        return doy
    if period == "WeekOfYear":
        jan1 = days - (doy - 1)
        return _fdiv(doy - 1 + day_of_week(jan1) - 1, 7) + 1
    if period == "WeekOfMonth":
        first = days - (d - 1)
        return _fdiv(d - 1 + day_of_week(first) - 1, 7) + 1
    raise ValueError(f"unknown time period {period}")


def period_values(ms: torch.Tensor, period: str, raw: bool = False):
    """(value, period size) as ``DateToUnitCircle.getPeriodWithSize`` (0-based when min == 1)."""
    lo, hi = TIME_PERIODS[period]
    v = fields(ms, period)
    if raw:
        return v, hi
    return (v - 1 if lo == 1 else v), hi


# ------------------------------------------------------------------- string helpers (DateTimeUtils.scala:40-142)
_FORMATS = ("%Y-%m-%d %H:%M:%S.%f", "%Y-%m-%d %H:%M:%S", "%Y/%m/%d", "%m/%d/%Y")


def parse(date: str, tz: str = "UTC") -> int:
    """``DateTimeUtils.parse``: epoch ms of ``yyyy-MM-dd HH:mm:ss.SSS``, ``yyyy-MM-dd HH:mm:ss``, ``yyyy/MM/dd``,
    ``M/d/yyyy`` or an ISO date-time, read in ``tz`` (UTC by default) unless the string carries an offset."""
    import datetime as dt
    from zoneinfo import ZoneInfo
    zone = dt.timezone.utc if tz in ("UTC", "GMT+0", "GMT") else ZoneInfo(tz)
    for f in _FORMATS:
        try:
            d = dt.datetime.strptime(date, f)
            break
        except ValueError:
            continue
    else:
        s = date[:-1] + "+00:00" if date.endswith("Z") else date
        try:
            d = dt.datetime.fromisoformat(s)
        except ValueError:
            raise ValueError(f"Invalid format: \"{date}\"") from None
    if d.tzinfo is None:
        d = d.replace(tzinfo=zone)
    return int(round(d.timestamp() * 1000))


def parse_unix(ms: int) -> str:
    """``DateTimeUtils.parseUnix``: the UTC ``yyyy/MM/dd`` of an epoch-ms timestamp."""
    import datetime as dt
    return dt.datetime.fromtimestamp(ms / 1000.0, dt.timezone.utc).strftime("%Y/%m/%d")


def get_standard_days(start_ms: int, end_ms: int) -> int:
    """``DateTimeUtils.getStandardDays``: whole days of ``end - start``, truncated toward zero."""
    d = int(end_ms) - int(start_ms)
    return d // MS_PER_DAY if d >= 0 else -((-d) // MS_PER_DAY)


def get_range(start: str, end: str):
    """``DateTimeUtils.getRange``: every ``yyyy/MM/dd`` from ``start`` to ``end`` inclusive."""
    s = parse(start)
    return [parse_unix(s + k * MS_PER_DAY) for k in range(get_standard_days(s, parse(end)) + 1)]


def get_date_plus_days(start: str, days: int) -> str:
    """``DateTimeUtils.getDatePlusDays``: ``start`` plus ``days`` calendar days, as ``yyyy/MM/dd``."""
    return parse_unix(parse(start) + int(days) * MS_PER_DAY)
