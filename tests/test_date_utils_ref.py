"""``DateTimeUtilsTest.scala`` ported: ISO and ``yyyy-MM-dd HH:mm:ss.SSS`` parsing, ``parseUnix``, the inclusive day
range over 500 days, and ``getDatePlusDays``; plus ``getStandardDays`` truncating toward zero."""
import datetime as dt

from transmogrifai_amd.utils import dates as D

UTC = dt.timezone.utc
DATE_STR = "2017-03-29T14:00:07.000Z"
DATE = dt.datetime(2017, 3, 29, 14, 0, 7, tzinfo=UTC)
MS = int(DATE.timestamp() * 1000)


def test_parse_iso_and_formatted():
    assert D.parse(DATE_STR) == MS
    assert D.parse("2017-03-29 14:00:07.000") == MS
    assert D.parse("2017/03/29") == int(dt.datetime(2017, 3, 29, tzinfo=UTC).timestamp() * 1000)
    assert D.parse("3/29/2017") == D.parse("2017/03/29")


def test_parse_unix():
    now = dt.datetime.now(UTC)
    assert D.parse_unix(int(now.timestamp() * 1000)) == now.strftime("%Y/%m/%d")


def test_range_between_two_dates():
    start = (DATE - dt.timedelta(days=500)).strftime("%Y/%m/%d")
    rng = D.get_range(start, DATE.strftime("%Y/%m/%d"))
    assert len(rng) == 501 and rng[0] == start and rng[-1] == "2017/03/29"


def test_date_plus_days():
    now = dt.datetime.now(UTC)
    assert D.get_date_plus_days(now.strftime("%Y/%m/%d"), 31) == (now + dt.timedelta(days=31)).strftime("%Y/%m/%d")


def test_standard_days_truncate():
    assert D.get_standard_days(0, 100 * D.MS_PER_DAY + 60_000) == 100
    assert D.get_standard_days(100 * D.MS_PER_DAY + 60_000, 0) == -100
