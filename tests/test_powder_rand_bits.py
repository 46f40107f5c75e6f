"""CPU: the integer form of the powderworld rand decision bits
(powder_full.h FullWorld::rand_bits_w, used on the Philox path) equals the
float32 form (FullWorld::rand_bits, the reference's comparisons, sim.py) for
every 24-bit uniform u01f_from(w) = (w >> 8) 2^-24 -- all 2^24 values of each
of the three fields.  The thresholds are read from the header."""

import os
import re

import numpy as np

HDR = os.path.join(os.path.dirname(__file__), '..', 'ogbench_amd', 'csrc', 'powder_full.h')


def _consts():
    text = open(HDR).read()
    out = {}
    for name, val in re.findall(r'(k(?:Rm|Ri|Re)\w+) = (\d+)u << 8', text):
        out[name] = int(val) << 8
    return out


def _float_bits(rm, ri, re):
    f = np.float32
    b = (rm > f(0.5)).astype(np.int64)
    for j in range(3):
        x = (rm + f(2 * j - 2)).astype(np.float32)
        b |= ((x + f(0.0)).astype(np.float32) > f(0.5)).astype(np.int64) << (1 + j)
        b |= ((x + f(2.0)).astype(np.float32) > f(0.5)).astype(np.int64) << (4 + j)
    ic = np.where(ri < f(0.02), 0, np.where(ri < f(0.05), 1, np.where(ri < f(0.2), 2, np.where(ri < f(0.3), 3, 4))))
    ec = np.where(re < f(0.05), 0, np.where(re < f(0.4), 1, 2))
    return b | (ic << 7) | (ec << 10)


def _int_bits(wm, wi, we, c):
    b = 0x68 | np.where(wm >= c['kRmHalf'], 0x5, 0) | np.where(wm >= c['kRmHalfR'], 0x10, 0)
    ic = sum((wi >= c[k]).astype(np.int64) for k in ('kRiT0', 'kRiT1', 'kRiT2', 'kRiT3'))
    ec = sum((we >= c[k]).astype(np.int64) for k in ('kReT0', 'kReT1'))
    return b | (ic << 7) | (ec << 10)


def test_integer_decision_bits_equal_float_bits():
    c = _consts()
    assert len(c) == 8
    k = np.arange(1 << 24, dtype=np.int64)
    u = (k.astype(np.float32) * np.float32(2.0 ** -24)).astype(np.float32)
    w_lo, w_hi = k << 8, (k << 8) | 0xFF  # both ends of each word range with the same (w >> 8)
    fb = _float_bits(u, u, u)
    for w in (w_lo, w_hi):
        assert np.array_equal(_int_bits(w, w, w, c), fb)
    # the three fields are independent: shifted pairings
    rng = np.random.RandomState(0)
    p = rng.permutation(1 << 24)
    assert np.array_equal(_int_bits(w_lo, w_lo[p], w_hi[::-1], c), _float_bits(u, u[p], u[::-1]))
