"""nGQL integer literals as the reference scanner reads them (src/parser/scanner.lex:328-368).

Pinned to ScannerTest.cpp:415-430 (values and lexical errors); the longest-match cases ("09",
"0789": flex prefers the longer {DEC}+ match over the shorter 0{OCT}+ one, first rule on a tie)
follow the scanner's rules directly.  CPU only."""
import pytest

from tests.support.ngql import ParseError, int_literal, parse

# ScannerTest.cpp:415-430 (int64 values: the sscanf conversions wrap)
PINNED = [("123", 123), ("0x123", 0x123), ("0xdeadbeef", 0xdeadbeef), ("0123", 0o123),
          ("0xFFFFFFFFFFFFFFFF", -1), ("0x00FFFFFFFFFFFFFFFF", -1),
          ("9223372036854775807", 9223372036854775807), ("001777777777777777777777", -1)]
PINNED_ERRORS = ["9223372036854775808", "0xFFFFFFFFFFFFFFFFF", "002777777777777777777777"]
# longest match / first rule on a tie (scanner.lex rule order: hex, octal, decimal)
DERIVED = [("0", 0), ("09", 9), ("0789", 789), ("0777", 0o777), ("00", 0), ("0x00000000000000001", 1)]


@pytest.mark.parametrize("text,value", PINNED + DERIVED)
def test_integer_literal_value(text, value):
    assert int_literal(text) == value
    # and through the statement parser (a GO start vid is an INTEGER token)
    assert parse(f"GO FROM {text} OVER like")[0].from_vids == [value]


@pytest.mark.parametrize("text", PINNED_ERRORS)
def test_integer_literal_lexical_error(text):
    with pytest.raises(ParseError):
        int_literal(text)
    with pytest.raises(ParseError):
        parse(f"GO FROM {text} OVER like")
