"""K3 wide rows (zipkin_amd/csrc/zk_reduce.hip, k_bucket_lds_reduce_wide): the 42-bit pieces and the
flush into the table's 32-bit limbs, restated in Python integers.

The table keeps each power sum S_k = sum d^k as u64 limbs of weight 2^(32 j), carry-free: the value is
sum limb_j * 2^(32 j), and finalize resolves the carries (zk_finalize.hip). It must hold up to 2^32 - 1
records since reset (zk_internal.h kMaxRecordsSinceReset) without a limb overflowing. These tests
check, for durations up to the largest accepted (2^40 - 1 us) and sub-parts up to 2^20 links:
  * every LDS row sum stays < 2^64 (the kernel's 64-bit LDS atomics);
  * the rebuilt S_k equals the exact sum and the limbs encode it;
  * every limb but the top one of a sum receives < 2^32 per flush, the top one at most
    sum over the flush's links of (floor(d^k / 2^(32 top)) + 1);
so after at most 2^32 - 1 links (each flush holding at least one) every limb stays < 2^64."""
import random

P42 = (1 << 42) - 1
M32 = (1 << 32) - 1
LIMB_BASE = {1: 1, 2: 3, 3: 6, 4: 10}  # kLimbS1..kLimbS4
LIMB_COUNT = {1: 2, 2: 3, 3: 4, 4: 5}
SUB = 1 << 20  # links per sub-part


def rows_of(ds):
    """The 12 LDS rows of one cell after adding the links `ds` (the kernel's per-link pieces)."""
    r = [0] * 12
    for d in ds:
        if d < (1 << 21):
            d2, d3, d4 = d * d, d ** 3, d ** 4
            r[11] += (1 << 42) | d
            r[2] += d2
            r[4] += d3 & P42
            r[5] += d3 >> 42
            r[7] += d4 & P42
            r[8] += d4 >> 42
        else:
            d2, d3, d4 = d * d, d ** 3, d ** 4
            r[0] += 1
            r[1] += d
            r[2] += d2 & P42
            r[3] += d2 >> 42
            r[4] += d3 & P42
            r[5] += (d3 >> 42) & P42
            r[6] += d3 >> 84
            r[7] += d4 & P42
            r[8] += (d4 >> 42) & P42
            r[9] += (d4 >> 84) & P42
            r[10] += d4 >> 126
    return r


def flush(r):
    """The kernel's rebuild of m0, S1..S4 and their cut into 15 limbs."""
    m0 = r[0] + (r[11] >> 42)
    s = {1: r[1] + (r[11] & P42),
         2: r[2] + (r[3] << 42),
         3: r[4] + (r[5] << 42) + (r[6] << 84),
         4: r[7] + (r[8] << 42) + (r[9] << 84) + (r[10] << 126)}
    limbs = [0] * 15
    limbs[0] = m0
    for k in (1, 2, 3, 4):
        base, cnt = LIMB_BASE[k], LIMB_COUNT[k]
        for j in range(cnt - 1):
            limbs[base + j] = (s[k] >> (32 * j)) & M32
        limbs[base + cnt - 1] = s[k] >> (32 * (cnt - 1))  # the top limb takes the rest
    return m0, s, limbs


def check(ds):
    r = rows_of(ds)
    assert all(0 <= x < (1 << 64) for x in r), "an LDS row overflowed"
    m0, s, limbs = flush(r)
    assert m0 == len(ds)
    for k in (1, 2, 3, 4):
        exact = sum(d ** k for d in ds)
        assert s[k] == exact
        base, cnt = LIMB_BASE[k], LIMB_COUNT[k]
        assert sum(limbs[base + j] << (32 * j) for j in range(cnt)) == exact
        for j in range(cnt - 1):
            assert limbs[base + j] <= M32
        top = cnt - 1
        assert limbs[base + top] <= sum((d ** k >> (32 * top)) + 1 for d in ds)
    # the per-link bound the 2^32 edge needs: every limb's share of one link is <= 2^32
    for d in (max(ds), 1):
        for k in (1, 2, 3, 4):
            assert (d ** k >> (32 * (LIMB_COUNT[k] - 1))) + 1 <= 1 << 32
    return limbs


def test_extreme_durations_one_subpart():
    dmax = (1 << 40) - 1
    for ds in ([dmax] * SUB, [(1 << 21) - 1] * SUB, [1 << 21] * SUB, [0] * 5, [dmax, 0, 1, (1 << 32) + 7]):
        # a sub-part of 2^20 equal links: exercise the row sums at their bound without 1M-term loops
        if len(ds) == SUB:
            d = ds[0]
            r = [x * SUB for x in rows_of([d])]
            assert all(x < (1 << 64) for x in r)
            m0, s, limbs = flush(r)
            for k in (1, 2, 3, 4):
                assert s[k] == SUB * d ** k
                base, cnt = LIMB_BASE[k], LIMB_COUNT[k]
                assert sum(limbs[base + j] << (32 * j) for j in range(cnt)) == SUB * d ** k
                assert all(limbs[base + j] <= M32 for j in range(cnt - 1))
        else:
            check(ds)


def test_random_mixes():
    rng = random.Random(7)
    for _ in range(200):
        n = rng.randint(1, 300)
        ds = [rng.choice([rng.randrange(1 << 21), rng.randrange(1 << 32), rng.randrange(1 << 40)]) for _ in range(n)]
        check(ds)


def test_table_limbs_hold_2_pow_32_minus_1_links():
    """Worst case over a whole job: 2^32 - 1 links (the records-since-reset bound) in one cell, every
    one in its own flush (the most flushes possible), at the largest duration: every limb total
    stays < 2^64."""
    links = (1 << 32) - 1
    dmax = (1 << 40) - 1
    _, _, one = flush(rows_of([dmax]))
    worst_non_top = M32  # < 2^32 per flush for every non-top limb
    for k in (1, 2, 3, 4):
        base, cnt = LIMB_BASE[k], LIMB_COUNT[k]
        for j in range(cnt - 1):
            assert one[base + j] <= worst_non_top
            assert worst_non_top * links < 1 << 64
        top_share = (dmax ** k >> (32 * (cnt - 1))) + 1
        assert top_share * links < 1 << 64
    assert links * 1 < 1 << 64  # m0
