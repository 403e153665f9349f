"""Host restatements of two shortcuts in the device sampler's integer and
comparison arithmetic (hb_mcmc_amd/csrc/hb_dsampler.hip). Neither needs a GPU.

1. ran2 jump-ahead. ds_propose gets the two L'Ecuyer LCG terms of draw k
   (mcmc_wrapper2.c:919-925, Schrage's method) lane-parallel as
   IA^(k+1) * z mod IM: a 62-bit product folded twice at 2^31 = c (mod 2^31 - c),
   then one conditional subtraction (mulmod31<C>). That must equal k+1 Schrage
   steps for every state the stream can reach.
2. Tempering test. ds_swap decides exp(x) >= beta (:803-806) as x >= ln(beta) + d
   (accept) or x <= ln(beta) - d (reject), with d = 1e-12 (1 + |ln beta|). Only
   inside that band, or for beta = 0 or NaN x, does it evaluate exp. The decision
   must equal libm's exp(x) >= beta. Python's math.exp/math.log are the host glibc
   functions the reference calls.
"""
import math

import numpy as np

IM1, IA1, IQ1, IR1 = 2147483563, 40014, 53668, 12211
IM2, IA2, IQ2, IR2 = 2147483399, 40692, 52774, 3791


def schrage(z, ia, iq, ir, im):  # mcmc_wrapper2.c:919-925 (C integer division truncates)
    k = z // iq if z >= 0 else -((-z) // iq)
    z = ia * (z - k * iq) - k * ir
    return z + im if z < 0 else z


def mulmod31(a, z, c):  # hb_dsampler.hip mulmod31<C>
    x = a * z
    x = (x >> 31) * c + (x & 0x7FFFFFFF)
    x = (x >> 31) * c + (x & 0x7FFFFFFF)
    r = x & 0xFFFFFFFF
    m = (1 << 31) - c
    return r - m if r >= m else r


def test_moduli_are_two_pow_31_minus_c():
    assert IM1 == (1 << 31) - 85 and IM2 == (1 << 31) - 249


def test_jump_ahead_equals_schrage_steps():
    rng = np.random.default_rng(20261016)
    for ia, iq, ir, im, c in ((IA1, IQ1, IR1, IM1, 85), (IA2, IQ2, IR2, IM2, 249)):
        pw, p = [], 1
        for _ in range(64):  # LcgPow: IA^(k+1) mod IM, k < 64
            p = p * ia % im
            pw.append(p)
        starts = [1, 2, im - 1, im - 2, iq, iq - 1, iq + 1] + [int(v) for v in rng.integers(1, im, 400)]
        for z0 in starts:
            z = z0
            for k in range(64):
                z = schrage(z, ia, iq, ir, im)
                assert mulmod31(pw[k], z0, c) == z, (im, z0, k)


def decide(x, beta):  # ds_swap's attempt(): band test, exact exp inside the band
    lnb = math.log(beta) if beta > 0 else -math.inf
    if lnb > -math.inf:
        d = 1e-12 * (1.0 + abs(lnb))
        if x >= lnb + d:
            return True
        if x <= lnb - d:
            return False
    return math.exp(x) >= beta if not math.isnan(x) else False


def test_swap_band_decision_equals_exp_compare():
    rng = np.random.default_rng(7)
    rand_max = 2147483647
    r = rng.integers(0, rand_max + 1, 20000)
    betas = [float(v) / rand_max for v in r] + [0.0, 1.0, 1.0 / rand_max]
    for beta in betas:
        lnb = math.log(beta) if beta > 0 else 0.0
        # far away, near the band edges, and at the exact boundary (ulp steps around ln beta)
        xs = [lnb - 5.0, lnb + 5.0, lnb, math.nextafter(lnb, math.inf), math.nextafter(lnb, -math.inf),
              lnb + 2e-12 * (1 + abs(lnb)), lnb - 2e-12 * (1 + abs(lnb)), -math.inf, math.inf, math.nan]
        for x in xs:
            ref = (math.exp(x) >= beta) if not math.isnan(x) else False
            assert decide(x, beta) == ref, (x, beta)
