"""TEST INFRASTRUCTURE ONLY — Moments arithmetic for the oracle.

Two restatements of the Moments the reference computes:

* `algebird_plus` / `algebird_fold`: the pairwise fp64 combine of algebird-core 0.8.1
  (`com.twitter.algebird.MomentsGroup.plus`, `Moments.getCombinedMean`; artifact
  com.twitter:algebird-core_2.10:0.8.1 pinned at project/Project.scala:42,50, not vendored in the
  reference, restated here from its published algorithm). The reference reaches it through
  `Moments(d.toDouble)` and `.group.sum` (ZipkinAggregateJob.scala:35,39-40) and through
  `DependencyLink.sg.plus` (Dependencies.scala:38-43).
* `exact_moments` / `moments_from_power_sums`: the same quantities computed in exact rational
  arithmetic and rounded once (Python's int/int division is correctly rounded), which is what the
  product's finalize kernel reproduces bit for bit.

Algebird's fold and the exact value agree to ~1e-14 relative on realistic data (its result depends
on the fold order), hence the 1e-9 tolerance against the reference in BASELINE.json.
"""
from __future__ import annotations

from fractions import Fraction
from typing import Iterable, NamedTuple

STABILITY_CONSTANT = 0.1


class Moments(NamedTuple):
    m0: int
    m1: float
    m2: float
    m3: float
    m4: float

    @staticmethod
    def of(value: float) -> "Moments":  # Moments(value)
        return Moments(1, float(value), 0.0, 0.0, 0.0)

    # accessors as in zipkin-web momentAnnotations.js:6-11 (a port of algebird's)
    @property
    def count(self) -> int:
        return self.m0

    @property
    def mean(self) -> float:
        return self.m1

    @property
    def variance(self) -> float:
        return self.m2 / self.m0

    @property
    def stddev(self) -> float:
        return self.variance ** 0.5

    @property
    def skewness(self) -> float:
        return (self.m0 ** 0.5) * self.m3 / (self.m2 ** 1.5)

    @property
    def kurtosis(self) -> float:
        return self.m0 * self.m4 / (self.m2 ** 2) - 3


ZERO = Moments(0, 0.0, 0.0, 0.0, 0.0)


def combined_mean(n: int, an: float, k: int, ak: float) -> float:
    if n < k:
        return combined_mean(k, ak, n, an)
    new = n + k
    if new == 0:
        return 0.0
    if new == n:
        return an
    scaling = float(k) / new
    if scaling < STABILITY_CONSTANT:
        return an + (ak - an) * scaling
    return (n * an + k * ak) / new


def algebird_plus(a: Moments, b: Moments) -> Moments:
    delta = b.m1 - a.m1
    n = a.m0 + b.m0
    if n == 0:
        return ZERO
    mean = combined_mean(a.m0, a.m1, b.m0, b.m1)
    na, nb = float(a.m0), float(b.m0)
    m2 = a.m2 + b.m2 + delta ** 2 * na * nb / n
    m3 = (
        a.m3
        + b.m3
        + delta ** 3 * na * nb * (na - nb) / float(n) ** 2
        + 3 * delta * (na * b.m2 - nb * a.m2) / n
    )
    m4 = (
        a.m4
        + b.m4
        + delta ** 4 * na * nb * (na ** 2 - na * nb + nb ** 2) / float(n) ** 3
        + 6 * delta ** 2 * (na ** 2 * b.m2 + nb ** 2 * a.m2) / float(n) ** 2
        + 4 * delta * (na * b.m3 - nb * a.m3) / n
    )
    return Moments(n, mean, m2, m3, m4)


def algebird_fold(values: Iterable[float]) -> Moments:
    acc = ZERO
    for v in values:
        acc = algebird_plus(acc, Moments.of(v))
    return acc


def moments_from_power_sums(n: int, s1: int, s2: int, s3: int, s4: int) -> Moments:
    """Exact central moments from integer power sums, each rounded once to fp64."""
    if n == 0:
        return ZERO
    m1 = Fraction(s1, n)
    m2 = Fraction(n * s2 - s1 * s1, n)
    m3 = Fraction(n * n * s3 - 3 * n * s1 * s2 + 2 * s1 ** 3, n * n)
    m4 = Fraction(n ** 3 * s4 - 4 * n * n * s1 * s3 + 6 * n * s1 * s1 * s2 - 3 * s1 ** 4, n ** 3)
    return Moments(n, float(m1), float(m2), float(m3), float(m4))


def exact_moments(values: Iterable[int]) -> Moments:
    vs = [int(v) for v in values]
    n = len(vs)
    return moments_from_power_sums(
        n, sum(vs), sum(v * v for v in vs), sum(v ** 3 for v in vs), sum(v ** 4 for v in vs)
    )


def rel_close(a: float, b: float, rtol: float = 1e-9, atol: float = 0.0) -> bool:
    return abs(a - b) <= max(atol, rtol * max(abs(a), abs(b)))


def moments_close(a: Moments, b: Moments, rtol: float = 1e-9, scale_floor: float = 1e-12) -> bool:
    """m0 exact; m1..m4 within `rtol` relative error (BASELINE.json: 1e-9 in fp64).

    A central moment can be ~0 relative to the data it is computed from (m3 of a symmetric sample,
    m2 of near-constant durations), where any fp64 fold loses its relative accuracy. Those are
    compared against an absolute floor `scale_floor * n * (|mean| + sd)^k` — the data's own scale —
    which is also the SURVEY A.2 step-6 rule (1e-9 * m2^1.5 / sqrt(n) for m3) made uniform.
    """
    if a.m0 != b.m0:
        return False
    if a.m0 == 0:
        return True
    sd = (max(a.m2, 0.0) / a.m0) ** 0.5
    scale = abs(a.m1) + sd
    return (
        rel_close(a.m1, b.m1, rtol)
        and rel_close(a.m2, b.m2, rtol, atol=scale_floor * a.m0 * scale ** 2)
        and rel_close(a.m3, b.m3, rtol, atol=scale_floor * a.m0 * scale ** 3)
        and rel_close(a.m4, b.m4, rtol, atol=scale_floor * a.m0 * scale ** 4)
    )
