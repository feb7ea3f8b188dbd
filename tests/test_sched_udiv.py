"""The scheduler's division by a float reciprocal (udiv_small, hl_encoder.hip):
exact for the quotients k_pipeline takes (picture, row, stream index) with the
reciprocal correctly rounded or 1 ulp off either way (v_rcp_f32 per task)."""
import numpy as np


def udiv_small(a, d, inv):
    # float32 product truncated toward zero, then one correction each way
    q = int(np.float32(np.float32(a) * inv))
    q -= 1 if q * d > a else 0
    q += 1 if (q + 1) * d <= a else 0
    return q


def test_udiv_small_exact_with_approximate_reciprocals():
    rng = np.random.default_rng(5)
    # divisors: MB row widths / MB counts of every geometry up to 4096x2304,
    # pictures per stream and stream counts up to 128
    divisors = sorted({*range(1, 257), *(w * h for w in (11, 22, 40, 45, 60, 80, 120, 256) for h in (9, 18, 34, 68, 144)),
                       *rng.integers(1, 1 << 16, 200).tolist()})
    one = np.float32(1.0)
    for d in divisors:
        exact = one / np.float32(d)
        invs = (np.nextafter(exact, np.float32(0)), exact, np.nextafter(exact, np.float32(2)))
        qmax = min((1 << 24) - 1, d * (1 << 20)) // d  # a < 2^24, quotient below 2^20
        qs = np.unique(np.concatenate([np.arange(0, min(qmax, 64)), rng.integers(0, qmax + 1, 64), [qmax]]))
        for q in qs.tolist():
            for a in (q * d, q * d + d - 1, q * d + int(rng.integers(0, d))):
                if a >= (1 << 24):
                    continue
                for inv in invs:
                    assert udiv_small(a, d, inv) == a // d, (a, d, float(inv))
