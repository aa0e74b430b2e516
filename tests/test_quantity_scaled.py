"""Sub-milli Quantities: pas_quantity_to_scaled / pas_quantity_decimals
against an independent restatement of resource.ParseQuantity's value with Python's decimal
module (k8s.io/apimachinery v0.22.2, not vendored in the reference; the reference holds no
sub-milli literal, so these cases are parity unpinned against the reference itself and pinned
against the published algorithm: the exact decimal, rounded away from zero to 9 fractional
digits when it takes the inf.Dec path, capped at 2^63 - 1)."""
import re
from decimal import ROUND_UP, Decimal, getcontext

import numpy as np
import pytest

import pas_amd

getcontext().prec = 80
SI = {"n": -9, "u": -6, "m": -3, "": 0, "k": 3, "M": 6, "G": 9, "T": 12, "P": 15, "E": 18}
CAP = Decimal(2**63 - 1)


def go_value(literal: str) -> Decimal:
    """The Quantity's exact value as ParseQuantity leaves it (decimal SI / exponent forms)."""
    body, exp = literal, 0
    if "e" in literal or "E" in literal:
        i = max(literal.find("e"), literal.find("E"))
        body, exp = literal[:i], int(literal[i + 1:])
    else:
        for suf in ("n", "u", "m", "k", "M", "G", "T", "P", "E"):
            if literal.endswith(suf):
                body, exp = literal[: -len(suf)], SI[suf]
                break
    v = Decimal(body).scaleb(exp)
    digits = body.lstrip("+-").replace(".", "").lstrip("0")
    frac = len(body.split(".")[1]) if "." in body else 0
    fast = 18 - len(body.lstrip("+-").split(".")[0].lstrip("0")) - frac >= 0 and exp - frac >= -9
    if not fast or len(digits) > 18:  # inf.Dec: round away from zero at 1e-9, cap
        v = v.quantize(Decimal("1e-9"), rounding=ROUND_UP) if v != 0 else v
        v = max(min(v, CAP), -CAP)
    return v


def want_decimals(v: Decimal) -> int:
    for k in range(10):
        if (v.scaleb(k)) == (v.scaleb(k)).to_integral_value():
            return k
    raise AssertionError(v)


CASES = ["1500u", "0.0005", "1e-7", "100n", "1.5m", "0.0015", "2k", "1.5", "-0.0005", "7n",
         "0.000000001", "123456.789012345", "-42.5u", "9e15", "1e-9", "3.25e-4", "0.5m",
         "999999999n", "12345678.9", "0", "-1n", "4.2E-3"]


@pytest.mark.parametrize("lit", CASES)
def test_decimals_and_scaled_match_decimal_restatement(lit):
    v = go_value(lit)
    k = want_decimals(v)
    assert pas_amd.quantity_decimals(lit) == k, lit
    for places in range(k, 10):
        want = int(v.scaleb(places))
        if -2**63 <= want < 2**63:
            assert pas_amd.quantity_to_scaled(lit, places) == want, (lit, places)
        else:
            with pytest.raises(pas_amd.PasError) as e:
                pas_amd.quantity_to_scaled(lit, places)
            assert e.value.code == pas_amd._lib.PAS_ENOTEXACT
    if k > 0:  # fewer places than the value has: not exact
        with pytest.raises(pas_amd.PasError) as e:
            pas_amd.quantity_to_scaled(lit, k - 1)
        assert e.value.code == pas_amd._lib.PAS_ENOTEXACT
    if k <= 3:
        assert pas_amd.quantity_to_milli(lit) == int(v.scaleb(3))


def test_inf_dec_rounds_away_from_zero_at_nano():
    # more than 9 fractional digits: the inf.Dec path rounds up to the next 1e-9
    assert pas_amd.quantity_decimals("0.0000000001") == 9
    assert pas_amd.quantity_to_scaled("0.0000000001", 9) == 1
    assert pas_amd.quantity_to_scaled("-0.0000000001", 9) == -1
    assert pas_amd.quantity_to_scaled("1.0000000001", 9) == 1_000_000_001


def test_random_literals():
    rng = np.random.default_rng(0x5AB)
    for _ in range(3000):
        frac = int(rng.integers(0, 10))
        ip = int(rng.integers(0, 10**int(rng.integers(0, 10))))
        fp = int(rng.integers(0, 10**frac)) if frac else 0
        sign = "-" if rng.random() < 0.2 else ""
        body = f"{sign}{ip}" + (f".{fp:0{frac}d}" if frac else "")
        suf = ["", "", "m", "u", "n", "k", f"e-{int(rng.integers(1, 4))}"][int(rng.integers(0, 7))]
        lit = body + suf
        v = go_value(lit)
        k = want_decimals(v)
        assert pas_amd.quantity_decimals(lit) == k, lit
        want = int(v.scaleb(k))
        if -2**63 <= want < 2**63:
            assert pas_amd.quantity_to_scaled(lit, k) == want, lit


def test_scaled_argument_errors():
    with pytest.raises(pas_amd.PasError):
        pas_amd.quantity_to_scaled("1", 10)
    with pytest.raises(pas_amd.PasError):
        pas_amd.quantity_to_scaled("1", -1)
    with pytest.raises(pas_amd.PasError):
        pas_amd.quantity_decimals("1.2.3")


GRAMMAR = re.compile(r"^[+-]?\d+(\.\d+)?([numkMGTP]|[eE][+-]?\d{1,2})?$")
ALPHABET = "0123456789.+-eEnumkMGTPKi \t"


@pytest.mark.parametrize("seed", range(4))
def test_mutated_literals(seed):
    """Random edits of valid literals (character swaps, cuts, inserts from the Quantity
    alphabet, binary suffixes): every call returns a value or PasError, and a literal in the
    plain decimal grammar (sign, digits, fraction, SI or exponent suffix) matches the decimal
    restatement (PAS_ENOTEXACT past int64)."""
    rng = np.random.default_rng(0x0F00 + seed)
    base = CASES + ["1Ki", "1.5Gi", "16Mi", "+7", "007", "-0", "1e18", "9.9e-10"]
    compared = 0
    for _ in range(3000):
        s = list(base[int(rng.integers(0, len(base)))])
        for _ in range(int(rng.integers(1, 4))):
            op = int(rng.integers(0, 3))
            i = int(rng.integers(0, len(s) + 1))
            ch = ALPHABET[int(rng.integers(0, len(ALPHABET)))]
            if op == 0 and s:
                s[min(i, len(s) - 1)] = ch
            elif op == 1 and s:
                del s[min(i, len(s) - 1)]
            else:
                s.insert(i, ch)
        lit = "".join(s)
        results = []
        for fn in (pas_amd.quantity_decimals, lambda x: pas_amd.quantity_to_scaled(x, 9),
                   pas_amd.quantity_to_milli):
            try:
                results.append(fn(lit))
            except pas_amd.PasError as e:
                results.append(e)
        if GRAMMAR.match(lit) and not ("e" in lit.lower() and lit[-1] in "EPTGMk"):
            v = go_value(lit)
            k = want_decimals(v)
            assert results[0] == k, lit
            want = int(v.scaleb(9))
            if -2**63 <= want < 2**63:
                assert results[1] == want, lit
            else:
                assert isinstance(results[1], pas_amd.PasError), lit
                assert results[1].code == pas_amd._lib.PAS_ENOTEXACT, lit
            compared += 1
    assert compared > 300
