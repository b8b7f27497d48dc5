"""Phone number validation and E.164 normalisation by region.

Reference: ``PhoneNumberParser`` (``core/.../stages/impl/feature/PhoneNumberParser.scala:254-330``), which defers to
Google libphonenumber (``PhoneNumberUtil.parse`` / ``isValidNumber`` / ``truncateTooLongNumber``) and picks the
region from a region-code or country-name feature (``validCountryCode``: international ``+`` numbers use the
generic region ``ZZ``, known region codes are used as given, anything else is matched to the closest
country name by Jaccard similarity of character bigrams).

libphonenumber's per-region metadata is not available here, so validation uses a compact numbering-plan
table: country calling code, national trunk prefix and the valid national-significant-number lengths per
region, with the North American Numbering Plan's area-code / exchange rules for the ``+1`` regions.
Parity with libphonenumber is therefore approximate (parity unpinned); the reference's own test vectors
(``PhoneNumberParserTest.scala``) are pinned in ``tests/test_phone.py``.
"""
from __future__ import annotations

import re
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

INTERNATIONAL_CODE = "ZZ"
DEFAULT_REGION = "US"
STRICT_VALIDATION = False

_NANP = ("US", "CA", "PR", "DO", "BS", "JM", "TT", "BB", "VI", "GU", "AG", "BM", "KY", "LC", "GD")

# region -> (calling code, trunk prefix, valid national significant number lengths)
_PLAN: Dict[str, Tuple[str, str, Tuple[int, ...]]] = {r: ("1", "1", (10,)) for r in _NANP}
_PLAN.update({
    "GB": ("44", "0", (9, 10)), "IE": ("353", "0", (7, 8, 9)), "FR": ("33", "0", (9,)),
    "DE": ("49", "0", tuple(range(6, 14))), "IT": ("39", "", tuple(range(6, 12))), "ES": ("34", "", (9,)),
    "PT": ("351", "", (9,)), "NL": ("31", "0", (9,)), "BE": ("32", "0", (8, 9)), "CH": ("41", "0", (9,)),
    "AT": ("43", "0", tuple(range(4, 14))), "SE": ("46", "0", tuple(range(7, 11))), "NO": ("47", "", (8,)),
    "DK": ("45", "", (8,)), "FI": ("358", "0", tuple(range(5, 13))), "PL": ("48", "", (9,)), "CZ": ("420", "", (9,)),
    "SK": ("421", "0", (9,)), "HU": ("36", "06", (8, 9)), "RO": ("40", "0", (9,)), "BG": ("359", "0", (8, 9)),
    "GR": ("30", "", (10,)), "TR": ("90", "0", (10,)), "RU": ("7", "8", (10,)), "UA": ("380", "0", (9,)),
    "IL": ("972", "0", (8, 9)), "SA": ("966", "0", (9,)), "AE": ("971", "0", (8, 9)), "EG": ("20", "0", (9, 10)),
    "ZA": ("27", "0", (9,)), "NG": ("234", "0", (8, 10)), "KE": ("254", "0", (9,)), "ZW": ("263", "0", (9,)),
    "CD": ("243", "0", (9,)), "MA": ("212", "0", (9,)), "IN": ("91", "0", (10,)), "PK": ("92", "0", (9, 10)),
    "BD": ("880", "0", (10,)), "CN": ("86", "0", (10, 11)), "HK": ("852", "", (8,)), "TW": ("886", "0", (8, 9)),
    "JP": ("81", "0", (9, 10)), "KR": ("82", "0", (9, 10)), "SG": ("65", "", (8,)), "MY": ("60", "0", (9, 10)),
    "TH": ("66", "0", (8, 9)), "VN": ("84", "0", (9, 10)), "PH": ("63", "0", (10,)), "ID": ("62", "0", (9, 10, 11)),
    "AU": ("61", "0", (9,)), "NZ": ("64", "0", (8, 9, 10)), "BR": ("55", "0", (10, 11)), "AR": ("54", "0", (10,)),
    "CL": ("56", "", (9,)), "CO": ("57", "", (10,)), "PE": ("51", "0", (8, 9)), "VE": ("58", "0", (10,)),
    "MX": ("52", "", (10,)), "AF": ("93", "0", (9,)), "IR": ("98", "0", (10,)), "IQ": ("964", "0", (10,)),
    "GH": ("233", "0", (9,)), "ET": ("251", "0", (9,)), "TZ": ("255", "0", (9,)), "UG": ("256", "0", (9,)),
    "DZ": ("213", "0", (8, 9)), "TN": ("216", "", (8,)), "LK": ("94", "0", (9,)), "NP": ("977", "0", (8, 10)),
    "IS": ("354", "", (7,)), "LU": ("352", "", tuple(range(4, 12))), "EE": ("372", "", (7, 8)), "LV": ("371", "", (8,)),
    "LT": ("370", "8", (8,)), "HR": ("385", "0", (8, 9)), "RS": ("381", "0", (8, 9)), "SI": ("386", "0", (8,)),
    "CY": ("357", "", (8,)), "MT": ("356", "", (8,)), "KZ": ("7", "8", (10,)),
})

# region -> country names (comma separated alternatives), the default codes-and-countries map
DEFAULT_COUNTRY_CODES: Dict[str, str] = {
    "US": "USA, United States of America", "CA": "Canada", "PR": "Puerto Rico", "DO": "Dominican Republic",
    "BS": "Bahamas", "JM": "Jamaica", "TT": "Trinidad and Tobago", "BB": "Barbados", "VI": "US Virgin Islands",
    "GU": "Guam", "AG": "Antigua and Barbuda", "BM": "Bermuda", "KY": "Cayman Islands", "LC": "Saint Lucia",
    "GD": "Grenada", "GB": "United Kingdom, Great Britain, England, UK", "IE": "Ireland", "FR": "France",
    "DE": "Germany", "IT": "Italy", "ES": "Spain", "PT": "Portugal", "NL": "Netherlands, Holland", "BE": "Belgium",
    "CH": "Switzerland", "AT": "Austria", "SE": "Sweden", "NO": "Norway", "DK": "Denmark", "FI": "Finland",
    "PL": "Poland", "CZ": "Czech Republic, Czechia", "SK": "Slovakia", "HU": "Hungary", "RO": "Romania",
    "BG": "Bulgaria", "GR": "Greece", "TR": "Turkey", "RU": "Russia, Russian Federation", "UA": "Ukraine",
    "IL": "Israel", "SA": "Saudi Arabia", "AE": "United Arab Emirates, UAE", "EG": "Egypt", "ZA": "South Africa",
    "NG": "Nigeria", "KE": "Kenya", "ZW": "Zimbabwe", "CD": "Democratic Republic of the Congo, Congo",
    "MA": "Morocco", "IN": "India", "PK": "Pakistan", "BD": "Bangladesh", "CN": "China", "HK": "Hong Kong",
    "TW": "Taiwan", "JP": "Japan", "KR": "South Korea, Korea", "SG": "Singapore", "MY": "Malaysia",
    "TH": "Thailand", "VN": "Vietnam", "PH": "Philippines", "ID": "Indonesia", "AU": "Australia",
    "NZ": "New Zealand", "BR": "Brazil", "AR": "Argentina", "CL": "Chile", "CO": "Colombia", "PE": "Peru",
    "VE": "Venezuela", "MX": "Mexico", "AF": "Afghanistan", "IR": "Iran", "IQ": "Iraq", "GH": "Ghana",
    "ET": "Ethiopia", "TZ": "Tanzania", "UG": "Uganda", "DZ": "Algeria", "TN": "Tunisia", "LK": "Sri Lanka",
    "NP": "Nepal", "IS": "Iceland", "LU": "Luxembourg", "EE": "Estonia", "LV": "Latvia", "LT": "Lithuania",
    "HR": "Croatia", "RS": "Serbia", "SI": "Slovenia", "CY": "Cyprus", "MT": "Malta", "KZ": "Kazakhstan",
}

SUPPORTED_REGIONS = frozenset(_PLAN)
_BY_CODE: Dict[str, List[str]] = {}
for _r, (_c, _, _) in _PLAN.items():
    _BY_CODE.setdefault(_c, []).append(_r)
_CLEAN = re.compile(r"[^+\d]")


def clean_number(pn: str) -> str:
    """``PhoneNumberParser.cleanNumber``: trim, keep only digits and ``+``."""
    return _CLEAN.sub("", pn.strip())


def _nanp_ok(nsn: str) -> bool:
    return len(nsn) == 10 and nsn[0] in "23456789" and nsn[3] in "23456789"


def _valid_nsn(nsn: str, region: str) -> bool:
    code, _, lengths = _PLAN[region]
    if code == "1":
        return _nanp_ok(nsn)
    return len(nsn) in lengths and nsn[0] != "0"


def _resolve(nsn: str, region: str, strict: bool) -> Optional[str]:
    """The valid national number (libphonenumber ``truncateTooLongNumber`` unless strict) or ``None``."""
    if _valid_nsn(nsn, region):
        return nsn
    if strict:
        return None
    lengths = (10,) if _PLAN[region][0] == "1" else _PLAN[region][2]
    for L in range(len(nsn) - 1, min(lengths) - 1, -1):     # drop trailing digits until valid
        if _valid_nsn(nsn[:L], region):
            return nsn[:L]
    return None


def parse(pn: Optional[str], region: str = DEFAULT_REGION, strict: bool = STRICT_VALIDATION) -> Optional[str]:
    """E.164 form ``+<code><national number>`` of a valid number, else ``None`` (``PhoneNumberParser.parse``);
    numbers shorter than 2 characters are ``None``."""
    if pn is None or len(pn) < 2:
        return None
    s = clean_number(pn)
    if not s or "+" in s[1:]:
        return None
    region = region.upper() if region else DEFAULT_REGION
    if s.startswith("+"):
        digits = s[1:]
        for k in (1, 2, 3):
            regs = _BY_CODE.get(digits[:k])
            if regs:
                nsn = _resolve(digits[k:], regs[0], strict)
                return None if nsn is None else f"+{digits[:k]}{nsn}"
        return None
    if region not in _PLAN:
        region = DEFAULT_REGION
    code, trunk, _ = _PLAN[region]
    digits = s
    cands = [digits]
    if trunk and digits.startswith(trunk):
        cands.append(digits[len(trunk):])
    if digits.startswith(code):
        cands.append(digits[len(code):])
    for c in cands:
        if _valid_nsn(c, region):
            return f"+{code}{c}"
    if strict:
        return None
    for c in cands:
        nsn = _resolve(c, region, False)
        if nsn is not None:
            return f"+{code}{nsn}"
    return None


def validate(pn: Optional[str], region: str = DEFAULT_REGION, strict: bool = STRICT_VALIDATION) -> Optional[bool]:
    """``PhoneNumberParser.validate``: ``None`` for a missing or < 2 character number, else validity."""
    if pn is None or len(pn) < 2:
        return None
    if "+" in clean_number(pn)[1:]:
        return None                     # unparseable (libphonenumber throws; the reference maps it to None)
    return parse(pn, region, strict) is not None


def _bigrams(s: str) -> set:
    s = s.strip()
    return {s[i:i + 2] for i in range(max(len(s) - 1, 1))} if s else set()


def _jaccard(a: set, b: set) -> float:
    u = len(a | b)
    return len(a & b) / u if u else 0.0


def valid_country_code(phone: Optional[str], region_text: Optional[str], default_region: str = DEFAULT_REGION,
                       region_codes: Sequence[str] = tuple(k.upper() for k in DEFAULT_COUNTRY_CODES),
                       country_names: Sequence[str] = tuple(v.upper() for v in DEFAULT_COUNTRY_CODES.values())
                       ) -> str:
    """``PhoneNumberParser.validCountryCode`` (PhoneNumberParser.scala:283-302)."""
    if phone is not None and phone.startswith("+"):
        return INTERNATIONAL_CODE
    if region_text is not None:
        rc = region_text.upper()
        if rc in region_codes:
            return rc
        if rc in SUPPORTED_REGIONS:
            return rc
        if region_codes:
            bi = _bigrams(rc)
            best, best_s = None, -1.0
            for code, names in zip(region_codes, country_names):
                for name in names.split(","):
                    sc = _jaccard(bi, _bigrams(name.strip()))
                    if sc > best_s:
                        best, best_s = code, sc
            return best
    return default_region


def validate_with_region(phone: Optional[str], region_text: Optional[str], default_region: str = DEFAULT_REGION,
                         strict: bool = STRICT_VALIDATION, codes_and_countries: Optional[Dict[str, str]] = None
                         ) -> Optional[bool]:
    """``IsValidPhoneNumber.transformFn``: region from the region feature, then :func:`validate`."""
    cc = codes_and_countries if codes_and_countries is not None else DEFAULT_COUNTRY_CODES
    code = valid_country_code(phone, region_text, default_region, [k.upper() for k in cc],
                              [v.upper() for v in cc.values()])
    return validate(phone, code if code != INTERNATIONAL_CODE else default_region, strict)


def parse_with_region(phone: Optional[str], region_text: Optional[str], default_region: str = DEFAULT_REGION,
                      strict: bool = STRICT_VALIDATION, codes_and_countries: Optional[Dict[str, str]] = None
                      ) -> Optional[str]:
    cc = codes_and_countries if codes_and_countries is not None else DEFAULT_COUNTRY_CODES
    code = valid_country_code(phone, region_text, default_region, [k.upper() for k in cc],
                              [v.upper() for v in cc.values()])
    return parse(phone, code if code != INTERNATIONAL_CODE else default_region, strict)


def check_codes(codes: Iterable[str]) -> None:
    """``setCodesAndCountries`` rejects region codes libphonenumber does not support."""
    bad = [c for c in codes if c.upper() not in SUPPORTED_REGIONS]
    if bad:
        raise ValueError(f"unsupported region codes: {bad}")
