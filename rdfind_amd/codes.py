"""Capture-code algebra and the capture-id layout used on the device.

Capture codes follow RDFind's bit layout (``ALG/util/ConditionCodes.scala:11-130``,
``ALG`` = ``rdfind-algorithm/src/main/scala/de/hpi/isg/sodap/rdfind``):
primary (condition) bits s=1, p=2, o=4 in bits 0-2 and the projection bit in
bits 3-5.  The nine valid standard captures are pinned by
``rdfind-algorithm/src/test/scala/.../ConditionCodes$Test.scala:28-33``.

On the device a capture is one ``uint32`` *capture id*:

* unary capture of type ``UNARY_CODES[t]`` with condition value ``v``
  -> ``t * V + v``  (``V`` = number of dictionary terms),
* binary capture with index ``b`` into the frequent-binary-condition table
  -> ``6 * V + b``.

The binary table stores ``(type, v1, v2)`` with ``v1`` belonging to the lowest
primary bit (``ConditionCodes.scala:70-79,95-100``).
"""
from __future__ import annotations

SUBJECT = 1
PREDICATE = 2
OBJECT = 4
NUM_TYPE_BITS = 3
TYPE_BIT_MASK = 7

_CHAR = {SUBJECT: "s", PREDICATE: "p", OBJECT: "o"}

# Unary capture codes, in the order used by the device id layout.
UNARY_CODES = (10, 12, 17, 20, 33, 34)  # s[p] s[o] p[s] p[o] o[s] o[p]
BINARY_CODES = (14, 21, 35)  # s[p,o] p[s,o] o[s,p]
ALL_CODES = UNARY_CODES + BINARY_CODES

UNARY_TYPE_INDEX = {c: i for i, c in enumerate(UNARY_CODES)}
BINARY_TYPE_INDEX = {c: i for i, c in enumerate(BINARY_CODES)}
UINT32_NONE = 0xFFFFFFFF


def lowest_one_bit(x: int) -> int:
    return x & -x


def bit_count(x: int) -> int:
    return bin(x & 0xFFFFFFFF).count("1")


def extract_primary(code: int) -> int:
    return code & TYPE_BIT_MASK


def extract_secondary(code: int) -> int:
    return (code >> NUM_TYPE_BITS) & TYPE_BIT_MASK


def create_code(first_primary: int, second_primary: int = 0, secondary: int = 0) -> int:
    """``ConditionCodes.createConditionCode`` (``ConditionCodes.scala:81-83``)."""
    return ((first_primary | second_primary) & TYPE_BIT_MASK) | ((secondary & TYPE_BIT_MASK) << NUM_TYPE_BITS)


def add_secondary(code: int) -> int:
    """``ConditionCodes.addSecondaryConditions`` (``ConditionCodes.scala:38-39``)."""
    return (code & TYPE_BIT_MASK) | ((~code & TYPE_BIT_MASK) << NUM_TYPE_BITS)


def is_binary(code: int) -> bool:
    return bit_count(code & TYPE_BIT_MASK) == 2


def is_unary(code: int) -> bool:
    return bit_count(code & TYPE_BIT_MASK) == 1


def is_subcode(candidate: int, super_code: int) -> bool:
    return (candidate & super_code) == candidate


def first_subcapture(code: int) -> int:
    """``ConditionCodes.extractFirstSubcapture`` (``ConditionCodes.scala:95``)."""
    return (code & ~TYPE_BIT_MASK) | lowest_one_bit(code)


def second_subcapture(code: int) -> int:
    """``ConditionCodes.extractSecondSubcapture`` (``ConditionCodes.scala:97-100``)."""
    first = lowest_one_bit(code)
    return (code & ~TYPE_BIT_MASK) | lowest_one_bit(code & ~first)


def decode(code: int):
    """``ConditionCodes.decodeConditionCode`` (``ConditionCodes.scala:70-79``)."""
    first = lowest_one_bit(code)
    second = lowest_one_bit(code & ~first)
    free = ~first & ~second & 7
    return first, second, free


def is_valid_standard_capture(code: int) -> bool:
    """``ConditionCodes.isValidStandardCapture`` (``ConditionCodes.scala:109-129``)."""
    primary = extract_primary(code)
    n_primary = bit_count(primary)
    if n_primary < 1 or n_primary > 2:
        return False
    secondary = extract_secondary(code)
    if bit_count(secondary) != 1:
        return False
    if primary & secondary:
        return False
    return (~0x3F & code) == 0


def pretty_print(code: int, value1: str, value2: str | None = None) -> str:
    """``ConditionCodes.prettyPrint`` (``ConditionCodes.scala:102-107``)."""
    proj = _CHAR.get(extract_secondary(code), "")
    first, second, _ = decode(extract_primary(code))
    if second == 0:
        return f"{proj}[{_CHAR[first]}={value1}]"
    return f"{proj}[{_CHAR[first]}={value1},{_CHAR[second]}={value2}]"


def format_cind(dep_code, dep_v1, dep_v2, ref_code, ref_v1, ref_v2, support) -> str:
    """``Cind.toString`` (``ALG/data/Cind.scala:29-31``)."""
    sup = "unknown support" if support == -1 else f"support={support}"
    return f"{pretty_print(dep_code, dep_v1, dep_v2)} < {pretty_print(ref_code, ref_v1, ref_v2)} ({sup})"


# ---------------------------------------------------------------------------
# Device capture-id layout helpers (host side).

def unary_capture_id(code: int, value: int, num_terms: int) -> int:
    return UNARY_TYPE_INDEX[code] * num_terms + value


def unary_components(code: int):
    """For a binary capture code, the two unary sub-capture codes (first, second)."""
    return first_subcapture(code), second_subcapture(code)
