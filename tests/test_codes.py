"""Port of the reference's unit tests that pin the capture-code alphabet and the null ordering:
rdfind-algorithm/src/test/scala/de/hpi/isg/sodap/rdfind/util/ConditionCodes$Test.scala:10-33 and
NullSensitiveOrdered$Test.scala:12-22."""
from rdfind_amd import codes
from oracle import rdfind_oracle as R

UNARY = [9, 10, 12, 17, 18, 20, 33, 34, 36]
BINARY = [11, 13, 14, 19, 21, 22, 35, 37, 38]


def test_is_binary_condition():  # ConditionCodes$Test.testIsBinaryCondition
    for c in UNARY:
        assert not codes.is_binary(c), c
        assert not R.is_binary(c), c
    for c in BINARY:
        assert codes.is_binary(c), c
        assert R.is_binary(c), c


def test_is_unary_condition():  # ConditionCodes$Test.testIsUnaryCondition
    for c in UNARY:
        assert codes.is_unary(c) and R.is_unary(c), c
    for c in BINARY:
        assert not codes.is_unary(c) and not R.is_unary(c), c


def test_sanity_check():  # ConditionCodes$Test.testSanityCheck
    all_codes = [10, 12, 17, 20, 33, 34, 14, 21, 35]
    for i in range(256):
        assert codes.is_valid_standard_capture(i) == (i in all_codes), i
    assert sorted(codes.ALL_CODES) == sorted(all_codes)


def test_null_sensitive_ordering():  # NullSensitiveOrdered$Test.testOrdering (via Condition.compare)
    k = lambda v: R.Cond(v, None, 10).key()  # noqa: E731
    assert k(None) <= k(None) and k(None) >= k(None)
    assert k("a") > k(None) and k(None) < k("a")
    assert k("a") >= k("a") and k("a") <= k("a")
    assert k("a") < k("b") and k("b") > k("a")


def test_subcaptures_and_pretty_print():
    # binary value1 belongs to the lowest primary bit (ConditionCodes.scala:70-79,95-107)
    assert codes.first_subcapture(35) == 33 and codes.second_subcapture(35) == 34
    assert codes.first_subcapture(21) == 17 and codes.second_subcapture(21) == 20
    assert codes.first_subcapture(14) == 10 and codes.second_subcapture(14) == 12
    assert codes.pretty_print(35, "<a>", "<b>") == "o[s=<a>,p=<b>]"
    assert codes.pretty_print(20, "<x>") == "p[o=<x>]"
    assert codes.format_cind(10, "<p>", None, 14, "<p>", "<o>", 3) == "s[p=<p>] < s[p=<p>,o=<o>] (support=3)"
    assert codes.add_secondary(3) == 35 and codes.add_secondary(5) == 21 and codes.add_secondary(6) == 14
