"""C-ABI checks that need no GPU: the library loads, exports every symbol include/pas.h
declares, and its host-only helpers (operator / Quantity parsing) behave as the
reference's call sites expect."""
import ctypes
import re

import pytest

import pas_amd
from pas_amd import _lib


def header_functions():
    with open(_lib.HEADER_PATH) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"\b(pas_[a-z0-9_]+)\s*\(", text))


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    declared = header_functions()
    assert len(declared) >= 20
    for name in sorted(declared):
        assert hasattr(lib, name), f"{name} declared in pas.h but not exported"
    # and the binding declares exactly the header's functions
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)


def test_abi_version():
    assert pas_amd.LIB.pas_abi_version() == 3


@pytest.mark.parametrize("op,want", [("LessThan", 0), ("GreaterThan", 1), ("Equals", 2),
                                     ("lessthan", -1), ("", -1), ("NotEquals", -1)])
def test_parse_operator(op, want):
    # core.EvaluateRule's operator map (operator.go:14-24) is case-sensitive
    assert pas_amd.parse_operator(op) == want


@pytest.mark.parametrize("q,milli", [
    ("10", 10_000), ("0", 0), ("-3", -3_000), ("+7", 7_000), ("100m", 100), ("2500m", 2500),
    ("1.5", 1500), (".5", 500), ("5.", 5000), ("1k", 1_000_000), ("1.5k", 1_500_000),
    ("1M", 10**9), ("1Ki", 1_024_000), ("1Mi", 1_048_576_000), ("0.5Ki", 512_000),
    ("1e3", 1_000_000), ("1E-3", 1), ("1000000u", 1000), ("1000000000n", 1000),
    ("9223372036854775.807", 2**63 - 1), ("-9223372036854775.808", -2**63),
])
def test_quantity_to_milli_exact(q, milli):
    assert pas_amd.quantity_to_milli(q) == milli


@pytest.mark.parametrize("q", ["1.0001", "1u", "1n", "0.0005", "9223372036854775.808",
                               "10P", "1Ei"])
def test_quantity_to_milli_not_exact(q):
    with pytest.raises(pas_amd.PasError) as e:
        pas_amd.quantity_to_milli(q)
    assert e.value.code == _lib.PAS_ENOTEXACT


@pytest.mark.parametrize("q", ["", "abc", "1x", "1.2.3", "--1", "1e", "1Kb"])
def test_quantity_unparsable(q):
    with pytest.raises(pas_amd.PasError) as e:
        pas_amd.quantity_to_milli(q)
    assert e.value.code == _lib.PAS_EINVAL


# resource.ParseQuantity (apimachinery v0.22.2) then AsInt64 with `ok` ignored
# (gpuscheduler/utils.go:23, scheduler.go:155), one case per parse path:
AS_INT64_CASES = [
    # int64Amount, scale 0
    ("2", 2), ("-1", -1), ("0", 0), ("00", 0), ("+7", 7), ("5.", 5), ("007", 7), ("-", 0),
    ("999999999999999999", 999999999999999999),            # 18 digits: precision 0
    # int64Amount, scale > 0: value * 10^scale, 0 on overflow
    ("2k", 2000), ("16G", 16 * 10**9), ("1e3", 1000), ("1E", 10**18), ("9E", 9 * 10**18),
    ("10E", 0), ("1e18", 10**18), ("1e19", 0), ("1.5k", 1500), ("1.0k", 1000),
    ("0.001k", 1), ("1e+3", 1000),
    # int64Amount, scale < 0: (0, false) even when the value is integral
    ("1.5", 0), ("500m", 0), ("1000m", 0), ("10.0", 0), ("1000000000n", 0), ("2000u", 0),
    ("1000e-3", 0), ("1.000000000", 0),
    # BinarySI fast path: precision = 15 - len(num) - exponent*3/10 - 1 >= 0
    ("8Gi", 8 * 2**30), ("1Ki", 1024), ("1023Ki", 1023 * 1024), ("1Ti", 2**40),
    ("10Ti", 10 * 2**40),
    # inf.Dec (precision < 0, or a fraction with a binary suffix, or scale < -9): 0
    ("100Ti", 0), ("1Pi", 0), ("1Ei", 0), ("123456789012Ki", 0), ("1.5Ki", 0),
    ("0.5Ki", 0), ("9223372036854775807", 0), ("1000000000000000000", 0),
    ("1.00000000000000000", 0), ("1e-10", 0),
    ("0000000000000000001", 1),                             # leading zeros do not count
]


@pytest.mark.parametrize("q,v", AS_INT64_CASES)
def test_quantity_as_int64(q, v):
    assert pas_amd.quantity_as_int64(q) == v


@pytest.mark.parametrize("q", ["", "1K", "abc", "1.2.3", "1e", "1Kb", "1ki"])
def test_quantity_as_int64_unparsable(q):
    with pytest.raises(pas_amd.PasError) as e:
        pas_amd.quantity_as_int64(q)
    assert e.value.code == _lib.PAS_EINVAL


@pytest.mark.parametrize("q,milli", [
    ("0.9999999999", 1000), ("-0.9999999999", -1000),  # inf.Dec: rounded away from 0 at 1n
    ("1.5Ki", 1_536_000), ("0.000000000", 0), ("-", 0),
])
def test_quantity_to_milli_parsed_value(q, milli):
    # the compared value is the parsed Quantity's (operator.go:16-22 CmpInt64 on it)
    assert pas_amd.quantity_to_milli(q) == milli


@pytest.mark.parametrize("q", ["1.0000000001", "1e-10", "9223372036854775808", "1e30", "1e-9"])
def test_quantity_to_milli_rounded_or_capped_not_exact(q):
    with pytest.raises(pas_amd.PasError) as e:
        pas_amd.quantity_to_milli(q)
    assert e.value.code == _lib.PAS_ENOTEXACT


def test_no_context_without_gpu_is_a_loud_error():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(pas_amd.PasError):
        pas_amd.Context(0)
