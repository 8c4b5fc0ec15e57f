"""commons-math3 3.4.1 MersenneTwister restated in Python (TEST INFRASTRUCTURE).

The reference's statistical tests draw their inputs from
org.apache.commons.math3.random.MersenneTwister (e.g.
T/UnivariateTimeSeriesSuite.scala:47-60 seeds 5 and 10,
T/models/AutoregressionSuite.scala:25-42 seed 10).  commons-math3 is a
third-party dependency (pom.xml:396-400) that is not vendored under
/root/reference, so its published algorithm is restated here:

* MersenneTwister(long seed) -> setSeed(int[]{(int)(seed>>>32), (int)seed})
  -> MT19937 init_by_array on top of setSeed(19650218);
* next(bits) = tempered MT19937 word >>> (32 - bits);
* BitsStreamGenerator.nextDouble() = ((long)next(26) << 26 | next(26)) * 2^-52
  (bit-exact: integer arithmetic only);
* BitsStreamGenerator.nextGaussian() = Box-Muller pair with a cached second
  deviate.  commons-math3 uses FastMath.log/cos/sin/sqrt; Python's libm can
  differ from FastMath in the last ulp, so Gaussian inputs match the
  reference's to ~1 ulp (irrelevant for the statistical tolerances 0.02-0.15
  those tests use).
"""
from __future__ import annotations

import math

N, M = 624, 397
MAG01 = (0x0, 0x9908B0DF)
MASK32 = 0xFFFFFFFF


class MersenneTwister:
    def __init__(self, seed: int):
        self.mt = [0] * N
        self.mti = N
        self._next_gaussian = math.nan
        self._set_seed_array([(seed >> 32) & MASK32, seed & MASK32])

    def _set_seed_int(self, seed: int):
        mt = self.mt
        mt[0] = seed & MASK32
        for i in range(1, N):
            mt[i] = (1812433253 * (mt[i - 1] ^ (mt[i - 1] >> 30)) + i) & MASK32
        self.mti = N
        self._next_gaussian = math.nan

    def _set_seed_array(self, seed):
        self._set_seed_int(19650218)
        mt = self.mt
        i, j = 1, 0
        for _ in range(max(N, len(seed))):
            l1 = mt[i - 1]
            mt[i] = ((mt[i] ^ ((l1 ^ (l1 >> 30)) * 1664525)) + seed[j] + j) & MASK32
            i += 1
            j += 1
            if i >= N:
                mt[0] = mt[N - 1]
                i = 1
            if j >= len(seed):
                j = 0
        for _ in range(N - 1):
            l1 = mt[i - 1]
            mt[i] = ((mt[i] ^ ((l1 ^ (l1 >> 30)) * 1566083941)) - i) & MASK32
            i += 1
            if i >= N:
                mt[0] = mt[N - 1]
                i = 1
        mt[0] = 0x80000000
        self._next_gaussian = math.nan

    def _twist(self):
        mt = self.mt
        for k in range(N):
            y = (mt[k] & 0x80000000) | (mt[(k + 1) % N] & 0x7FFFFFFF)
            mt[k] = mt[(k + M) % N] ^ (y >> 1) ^ MAG01[y & 1]
        self.mti = 0

    def next(self, bits: int) -> int:
        if self.mti >= N:
            self._twist()
        y = self.mt[self.mti]
        self.mti += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return (y & MASK32) >> (32 - bits)

    def next_double(self) -> float:
        high = self.next(26) << 26
        low = self.next(26)
        return float(high | low) * 2.0 ** -52

    def next_gaussian(self) -> float:
        if math.isnan(self._next_gaussian):
            x = self.next_double()
            y = self.next_double()
            alpha = 2 * math.pi * x
            r = math.sqrt(-2 * math.log(y))
            self._next_gaussian = r * math.sin(alpha)
            return r * math.cos(alpha)
        g = self._next_gaussian
        self._next_gaussian = math.nan
        return g
