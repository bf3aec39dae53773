"""Host view of the exact link accumulator (zk_config.table / zk_deps_partial).

The device accumulator is S*S cells x 16 u64 limbs (zipkin_amd/csrc/zk_internal.h): limb 0 is
m0 = n; limbs 1-2, 3-5, 6-9, 10-14 hold S1 = sum d, S2 = sum d^2, S3 = sum d^3, S4 = sum d^4 as
sums of 32-bit chunks, i.e. S_k = sum_i limb[off_k + i] << (32 i). The representation is linear
and carry-free below 2^32 records, so tables of disjoint traceId shards add limb-wise (what the
RCCL SUM all-reduce of the multi-GPU step does) and decode to the exact power sums of the union.

These helpers decode a table to exact integers on the host (for inspection, persistence of
incremental runs and the multi-process tests) and encode exact sums back into limbs.
"""
from __future__ import annotations

import numpy as np

LIMBS = 16
# (offset, number of 32-bit-weighted limbs) of S1..S4; mirrors kLimbS1..kLimbS4 in zk_internal.h
POWER_LIMBS = ((1, 2), (3, 3), (6, 4), (10, 5))
_M32 = (1 << 32) - 1


def decode_cell(limbs) -> tuple[int, int, int, int, int]:
    """(n, S1, S2, S3, S4) as exact Python ints from one cell's 16 limbs (any int/uint dtype)."""
    v = [int(x) & ((1 << 64) - 1) for x in limbs]
    sums = []
    for off, k in POWER_LIMBS:
        sums.append(sum(v[off + i] << (32 * i) for i in range(k)))
    return (v[0], *sums)


def decode(table: np.ndarray, num_services: int) -> dict:
    """{(parent, child): (n, S1, S2, S3, S4)} for every cell with n > 0."""
    t = np.asarray(table).reshape(num_services * num_services, LIMBS).view(np.uint64)
    out = {}
    for c in np.flatnonzero(t[:, 0]):
        out[(int(c // num_services), int(c % num_services))] = decode_cell(t[c])
    return out


def encode_cell(n: int, s1: int, s2: int, s3: int, s4: int) -> np.ndarray:
    """16 limbs (uint64) holding exact sums in the device layout (top limb takes the rest)."""
    out = np.zeros(LIMBS, np.uint64)
    out[0] = n
    for (off, k), s in zip(POWER_LIMBS, (s1, s2, s3, s4)):
        for i in range(k):
            chunk = (s >> (32 * i)) if i == k - 1 else ((s >> (32 * i)) & _M32)
            if chunk >= 1 << 64:
                raise OverflowError("power sum exceeds the accumulator's range")
            out[off + i] = chunk
    return out


def encode(sums: dict, num_services: int) -> np.ndarray:
    """Dense S*S*16 int64 table (the device dtype) from {(parent, child): (n, S1..S4)}."""
    t = np.zeros((num_services * num_services, LIMBS), np.uint64)
    for (p, c), v in sums.items():
        t[p * num_services + c] = encode_cell(*v)
    return t.reshape(-1).view(np.int64)
