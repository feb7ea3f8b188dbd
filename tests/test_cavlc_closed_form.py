"""The closed forms of hl_quad.h's quad_cavlc fast path, checked against the
per-coefficient formulation they replaced (and which the GPU parity tests
pin to the reference): on random 16-entry level lists, (a) the slow-path
test "any nonzero magnitude above 3" equals "a coded (non-trailing-one)
level above 3", (b) the level bits of the fast path equal
(sum of magnitudes + TotalCoeff) - 2 * trailing ones with the first coded
level's own length in place of its magnitude + 1, (c) the first coded level
sits at the highest coefficient above magnitude 1 unless more than three
trailing ones precede it.  (The CAVLC statistics themselves are the
reference's residual.c:587-901; cavlc_stat in hl_prims.h restates them.)"""
import random


def popc(x):
    return bin(x & 0xFFFFFFFF).count("1")


def clz(x):
    x &= 0xFFFFFFFF
    return 32 if x == 0 else 32 - x.bit_length()


def masks(levels):
    nz = ones = 0
    for i, lv in enumerate(levels):
        if lv:
            nz |= 1 << i
            ones |= (abs(lv) == 1) << i
    tc = popc(nz)
    hb = 31 - clz(nz & ~ones)
    t1a = popc(nz >> (hb + 1)) if hb + 1 < 32 else 0
    return nz, tc, hb, t1a, min(t1a, 3)


def per_coefficient(levels):
    """The former per-coefficient fast path: (slow, level bits)."""
    nz, tc, hb, t1a, t1 = masks(levels)
    sl0 = 1 if (tc > 10 and t1 < 3) else 0
    bits, slow = 0, False
    for i, lv in enumerate(levels):
        if not lv:
            continue
        m = popc(nz >> (i + 1)) - t1
        code = 2 * lv - 2 if lv > 0 else -2 * lv - 1
        if m == 0 and t1 < 3 and code >= 2:
            code -= 2
        if m >= 0:
            slow = slow or abs(lv) > 3
            bits += code + 1 if (m == 0 and sl0 == 0) else (code >> 1) + 2
    return slow, bits


def first_level_position(levels):
    """The first coded level: strip the t1 trailing ones from the top."""
    nz, tc, hb, t1a, t1 = masks(levels)
    rest = nz
    for _ in range(t1):
        rest &= ~(1 << ((31 - clz(rest)) & 31))
    return 31 - clz(rest) if rest else -1


def closed_form(levels):
    nz, tc, hb, t1a, t1 = masks(levels)
    sl0 = 1 if (tc > 10 and t1 < 3) else 0
    rest = nz
    for _ in range(3):
        rest &= ~(1 << ((31 - clz(rest)) & 31))
    pf = hb if t1a <= 3 else 31 - clz(rest)
    lf = levels[pf] if pf >= 0 else 0
    code = 2 * lf - 2 if lf > 0 else -2 * lf - 1
    if t1 < 3 and code >= 2:
        code -= 2
    lenf = code + 1 if sl0 == 0 else (code >> 1) + 2
    bits = sum(abs(v) for v in levels) + tc - 2 * t1 + (lenf - (abs(lf) + 1) if tc > t1 else 0)
    return any(abs(v) > 3 for v in levels), bits, pf


def test_closed_form_matches_per_coefficient():
    rng = random.Random(1)
    fast = 0
    for _ in range(40000):
        levels = [0] * 16
        for p in rng.sample(range(16), rng.randint(0, 16)):
            levels[p] = rng.choice([1, -1, 1, -1, 1, -1, 2, -2, 3, -3] + ([4, -5, 9] if rng.random() < 0.1 else []))
        slow, bits = per_coefficient(levels)
        slow2, bits2, pf = closed_form(levels)
        assert slow == slow2, levels
        assert pf == first_level_position(levels), levels
        if not slow:
            fast += 1
            assert bits == bits2, levels
    assert fast > 20000
