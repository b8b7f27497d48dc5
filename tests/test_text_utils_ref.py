"""``TextUtilsTest.scala`` ported: ``concat`` with empty halves, and ``cleanString`` / ``cleanOptString`` on a
string with special characters."""
from transmogrifai_amd.features.aggregators import concat_text
from transmogrifai_amd.utils.text import clean_opt, clean_string

BAD = "A string wit#h %bad pun&ctuation mark<=>s"


def test_concat():
    assert concat_text("Left", "Right", ",") == "Left,Right"
    assert concat_text("", "Right", ",") == "Right"
    assert concat_text("Left", "", ",") == "Left"
    assert concat_text("", "", ",") == ""


def test_clean_string_and_option():
    assert clean_string(BAD) == "AStringWitHBadPunCtuationMarkS"
    assert clean_opt(BAD) == "AStringWitHBadPunCtuationMarkS"
    assert clean_opt(None) is None
