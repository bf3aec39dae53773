"""Host view of the exact link accumulator (zk_config.table / zk_deps_partial).

The device accumulator is S*S cells x 16 u64 limbs (zipkin_amd/csrc/zk_internal.h): limb 0 is
m0 = n; limbs 1-2, 3-5, 6-9, 10-14 hold S1 = sum d, S2 = sum d^2, S3 = sum d^3, S4 = sum d^4 as
sums of 32-bit chunks, i.e. S_k = sum_i limb[off_k + i] << (32 i). The representation is linear
and carry-free below 2^32 records, so tables of disjoint traceId shards add limb-wise (what the
RCCL SUM all-reduce of the multi-GPU step does) and decode to the exact power sums of the union.

These helpers decode a table to exact integers on the host (for inspection, persistence of
incremental runs and the multi-process tests) and encode exact sums back into limbs.

The exchange form (zk_deps_partial, zipkin_amd/csrc/zk_exchange.hip) is what ranks all-reduce: 12
limbs of 56 bits per cell -- m0, S1 in two, S2 in two, S3 in three, S4 in four, each sum's top limb
holding its remaining bits -- so that a SUM over up to 256 ranks cannot carry out of a u64.
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


TAIL = 16  # counter words after the cells (zk_deps_partial: the folded zk_stats, in field order)


def decode(table: np.ndarray, num_services: int) -> dict:
    """{(parent, child): (n, S1, S2, S3, S4)} for every cell with n > 0 (the counter tail, if
    present, is ignored: see `tail_stats`)."""
    cells = num_services * num_services
    t = np.asarray(table).reshape(-1)[: cells * LIMBS].reshape(cells, LIMBS).view(np.uint64)
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


def encode(sums: dict, num_services: int, stats: dict | None = None) -> np.ndarray:
    """Dense int64 table in the device layout (S*S*16 limbs + the 16-word counter tail) from
    {(parent, child): (n, S1..S4)} and optional zk_stats counters."""
    t = np.zeros((num_services * num_services, LIMBS), np.uint64)
    for (p, c), v in sums.items():
        t[p * num_services + c] = encode_cell(*v)
    tail = np.zeros(TAIL, np.uint64)
    if stats:
        for i, k in enumerate(STAT_FIELDS):
            tail[i] = stats.get(k, 0)
    return np.concatenate([t.reshape(-1), tail]).view(np.int64)


# zk_stats field order = the device counter slots (zk_internal.h Stat), as folded into the tail
STAT_FIELDS = ("records", "merged_spans", "valid_spans", "invalid_spans", "child_spans", "joined_links",
               "missing_parent", "no_service", "ambiguous", "spilled_traces", "duration_range", "service_range",
               "trace_too_large")
_NOT_CLUSTERED_SLOT = 15


def tail_stats(table: np.ndarray, num_services: int, limbs: int = LIMBS) -> dict:
    """zk_stats counters from the tail of an accumulator (limbs = 16) or of the exchange buffer
    zk_deps_partial returns (limbs = XLIMBS)."""
    cells = num_services * num_services
    tail = np.asarray(table).reshape(-1)[cells * limbs : cells * limbs + TAIL].view(np.uint64)
    out = {k: int(tail[i]) for i, k in enumerate(STAT_FIELDS)}
    out["not_clustered"] = int(tail[_NOT_CLUSTERED_SLOT])
    return out


# ---- exchange form (zk_exchange.hip): 12 limbs of 56 bits per cell ---------------------------------
XLIMBS = 12
# (offset, limbs) of S1..S4 in the exchange cell (m0 is limb 0)
XPOWER_LIMBS = ((1, 2), (3, 2), (5, 3), (8, 4))
_M56 = (1 << 56) - 1


def encode_exchange_cell(n: int, s1: int, s2: int, s3: int, s4: int) -> np.ndarray:
    out = np.zeros(XLIMBS, np.uint64)
    out[0] = n
    for (off, k), s in zip(XPOWER_LIMBS, (s1, s2, s3, s4)):
        for i in range(k):
            x = (s >> (56 * i)) if i == k - 1 else ((s >> (56 * i)) & _M56)
            if x >= 1 << 64:
                raise OverflowError("power sum exceeds the exchange form's range")
            out[off + i] = x
    return out


def decode_exchange_cell(limbs) -> tuple[int, int, int, int, int]:
    v = [int(x) & ((1 << 64) - 1) for x in limbs]
    return (v[0], *(sum(v[off + i] << (56 * i) for i in range(k)) for off, k in XPOWER_LIMBS))


def encode_exchange(sums: dict, num_services: int, stats: dict | None = None) -> np.ndarray:
    """Dense int64 exchange buffer (S*S*12 limbs + the counter tail) from exact sums."""
    t = np.zeros((num_services * num_services, XLIMBS), np.uint64)
    for (p, c), v in sums.items():
        t[p * num_services + c] = encode_exchange_cell(*v)
    tail = np.zeros(TAIL, np.uint64)
    if stats:
        for i, k in enumerate(STAT_FIELDS):
            tail[i] = stats.get(k, 0)
    return np.concatenate([t.reshape(-1), tail]).view(np.int64)


def decode_exchange(x: np.ndarray, num_services: int) -> dict:
    cells = num_services * num_services
    t = np.asarray(x).reshape(-1)[: cells * XLIMBS].reshape(cells, XLIMBS).view(np.uint64)
    return {(int(c // num_services), int(c % num_services)): decode_exchange_cell(t[c]) for c in np.flatnonzero(t[:, 0])}


def pack(table: np.ndarray, num_services: int) -> np.ndarray:
    """Host restatement of k_table_pack: accumulator layout -> exchange form (tail copied)."""
    cells = num_services * num_services
    flat = np.asarray(table).reshape(-1)
    t = flat[: cells * LIMBS].reshape(cells, LIMBS).view(np.uint64)
    out = np.zeros((cells, XLIMBS), np.uint64)
    for c in range(cells):
        if t[c].any():
            out[c] = encode_exchange_cell(*decode_cell(t[c]))
    return np.concatenate([out.reshape(-1), flat[cells * LIMBS: cells * LIMBS + TAIL].view(np.uint64)]).view(np.int64)


def unpack(x: np.ndarray, num_services: int) -> np.ndarray:
    """Host restatement of k_table_unpack: exchange form -> accumulator layout (tail copied)."""
    cells = num_services * num_services
    flat = np.asarray(x).reshape(-1)
    t = flat[: cells * XLIMBS].reshape(cells, XLIMBS).view(np.uint64)
    out = np.zeros((cells, LIMBS), np.uint64)
    for c in range(cells):
        if t[c].any():
            out[c] = encode_cell(*decode_exchange_cell(t[c]))
    return np.concatenate([out.reshape(-1), flat[cells * XLIMBS: cells * XLIMBS + TAIL].view(np.uint64)]).view(np.int64)
