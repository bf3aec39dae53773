"""CPU restatement of the key-value popularity sketch (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module, as the
checker. It restates, in numpy, what include/zksketch.h promises for
Aggregates.getTopKeyValueAnnotations (zipkin-common/.../storage/Aggregates.scala:34):

  * per service a count-min sketch (Cormode & Muthukrishnan 2005) of `depth` rows x `width`
    counters; with h = mix64(k ^ seed_0), seed_0 = mix64(seed + 0x9E3779B97F4A7C15) and mix64 the
    splitmix64 finalizer, row r of key k is the top log2(width) bits of the 32-bit
    h1 + r * h2 (h1 = low half of h, h2 = high half | 1: double hashing, Kirsch & Mitzenmacher);
  * per service the best `candidates` keys, ordered by (estimate desc, key asc); after every
    batch the list is the best among (previous list U this batch's distinct keys), all estimated
    with the counters including the batch.

Parity of the product against this restatement is exact (same integers); the sketch's contract
against the exact counts (`exact_counts`) is the count-min bound, checked separately. The
reference itself has no producer for this list any more (CHANGELOG:7-8): there is no reference
output to pin it against ("parity unpinned" against the reference; pinned to the exact counts by
the error bound).
"""
from __future__ import annotations

import numpy as np

M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15


def mix64(z):
    """splitmix64 finalizer on a uint64 numpy array (wrapping arithmetic) or a Python int."""
    if isinstance(z, (int, np.integer)):
        z = int(z) & M64
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def auto_width(S: int) -> int:
    w = 1 << ((1 << 20) // S).bit_length() - 1 if (1 << 20) // S > 0 else 1
    return int(min(max(w, 64), 4096))


class KvOracle:
    def __init__(self, num_services: int, width: int = 0, depth: int = 4, candidates: int = 64, seed: int = 0):
        self.S = num_services
        self.width = width or auto_width(num_services)
        self.depth = depth
        self.cand = candidates
        self.wbits = self.width.bit_length() - 1
        self.seeds = [mix64((seed + GOLDEN * (r + 1)) & M64) for r in range(depth)]
        self.cm = np.zeros((self.S, depth, self.width), np.uint64)
        self.totals = np.zeros(self.S, np.uint64)
        self.lists: list[list[tuple[int, int]]] = [[] for _ in range(self.S)]
        self.dropped = 0

    def rows(self, keys: np.ndarray) -> np.ndarray:
        """[depth, n] counter index of every key in every row."""
        keys = np.asarray(keys, dtype=np.uint64)
        h = mix64(keys ^ np.uint64(self.seeds[0]))
        h1 = h & np.uint64(0xFFFFFFFF)
        h2 = (h >> np.uint64(32)) | np.uint64(1)
        sh = np.uint64(32 - self.wbits)
        with np.errstate(over="ignore"):
            return np.stack([(((h1 + np.uint64(r) * h2) & np.uint64(0xFFFFFFFF)) >> sh).astype(np.int64)
                             for r in range(self.depth)])

    def estimate(self, service: int, keys) -> np.ndarray:
        keys = np.asarray(keys, dtype=np.uint64)
        if len(keys) == 0:
            return np.zeros(0, np.uint64)
        idx = self.rows(keys)
        return np.min(np.stack([self.cm[service, r, idx[r]] for r in range(self.depth)]), axis=0)

    def accumulate(self, service_id, key_hash) -> None:
        svc = np.asarray(service_id, dtype=np.uint32)
        keys = np.asarray(key_hash).view(np.uint64) if np.asarray(key_hash).dtype == np.int64 else \
            np.asarray(key_hash, dtype=np.uint64)
        ok = svc < self.S
        self.dropped += int((~ok).sum())
        svc, keys = svc[ok].astype(np.int64), keys[ok]
        idx = self.rows(keys)
        for r in range(self.depth):
            np.add.at(self.cm[:, r, :], (svc, idx[r]), np.uint64(1))
        np.add.at(self.totals, svc, np.uint64(1))
        order = np.lexsort((keys, svc))
        svc_s, keys_s = svc[order], keys[order]
        bounds = np.flatnonzero(np.diff(svc_s)) + 1
        starts = np.concatenate([[0], bounds]) if len(svc_s) else np.zeros(0, np.int64)
        ends = np.concatenate([bounds, [len(svc_s)]]) if len(svc_s) else np.zeros(0, np.int64)
        touched = {}
        for a, b in zip(starts, ends):
            touched[int(svc_s[a])] = np.unique(keys_s[a:b])
        for s in range(self.S):
            new = touched.get(s)
            prev = np.array([k for k, _ in self.lists[s]], dtype=np.uint64)
            if new is None and len(prev) == 0:
                continue
            allk = np.unique(np.concatenate([prev, new])) if new is not None else prev
            est = self.estimate(s, allk)
            o = np.lexsort((allk, -est.astype(np.int64)))[: self.cand]
            self.lists[s] = [(int(allk[i]), int(est[i])) for i in o]

    @classmethod
    def merged(cls, shards: list["KvOracle"]) -> "KvOracle":
        """The job-wide sketch of disjoint item shards (include/zksketch.h, zk_kv_merge_candidates):
        counters and totals are summed (count-min is linear, so they equal one sketch over all
        items); every shard's list is offered, deduplicated, re-estimated against the summed
        counters and the best `candidates` kept, ordered (estimate desc, key asc)."""
        a = shards[0]
        out = cls(a.S, width=a.width, depth=a.depth, candidates=a.cand)
        out.seeds = list(a.seeds)
        out.cm = np.sum([o.cm for o in shards], axis=0, dtype=np.uint64)
        out.totals = np.sum([o.totals for o in shards], axis=0, dtype=np.uint64)
        out.dropped = sum(o.dropped for o in shards)
        for s in range(a.S):
            allk = np.unique(np.array([k for o in shards for k, _ in o.lists[s]], dtype=np.uint64))
            if len(allk) == 0:
                continue
            est = out.estimate(s, allk)
            o = np.lexsort((allk, -est.astype(np.int64)))[: out.cand]
            out.lists[s] = [(int(allk[i]), int(est[i])) for i in o]
        return out

    def topk(self, service: int, k: int) -> list[tuple[int, int]]:
        return self.lists[service][:k]

    def topk_all(self, k: int):
        keys = np.zeros((self.S, k), np.uint64)
        est = np.zeros((self.S, k), np.uint32)
        cnt = np.zeros(self.S, np.uint32)
        for s in range(self.S):
            lst = self.lists[s][:k]
            cnt[s] = len(lst)
            for i, (kk, e) in enumerate(lst):
                keys[s, i] = kk
                est[s, i] = e
        return keys, est, cnt


def exact_counts(service_id, key_hash, num_services: int) -> list[dict]:
    """Exact per-service key counts (the reference quantity the sketch approximates)."""
    svc = np.asarray(service_id, dtype=np.uint32)
    keys = np.asarray(key_hash).view(np.uint64) if np.asarray(key_hash).dtype == np.int64 else \
        np.asarray(key_hash, dtype=np.uint64)
    out: list[dict] = [dict() for _ in range(num_services)]
    ok = svc < num_services
    pairs = np.stack([svc[ok].astype(np.uint64), keys[ok]], 1)
    if len(pairs) == 0:
        return out
    u, c = np.unique(pairs, axis=0, return_counts=True)
    for (s, k), n in zip(u, c):
        out[int(s)][int(k)] = int(n)
    return out


def zipf_items(n: int, num_services: int, num_keys: int = 1_000_000, s: float = 1.1, seed: int = 4,
               key_salt: int = 0x5EED):
    """C4-shaped items: services uniform, key ranks Zipf(s) over num_keys ids, keys = mix64(rank)."""
    rng = np.random.default_rng(seed)
    w = 1.0 / np.arange(1, num_keys + 1, dtype=np.float64) ** s
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    rank = np.searchsorted(cdf, rng.random(n), side="right").astype(np.uint64)
    keys = mix64(rank + np.uint64(key_salt))
    svc = rng.integers(0, num_services, size=n, dtype=np.uint32)
    return svc, keys


class KvPortResult:
    def __init__(self, cm, totals, keys, est, cnt, dropped, seconds, threads):
        self.cm, self.totals, self.keys, self.est, self.cnt = cm, totals, keys, est, cnt
        self.dropped, self.seconds, self.threads = dropped, seconds, threads

    def topk_all(self, k: int):
        """(keys uint64[S, k], est uint32[S, k], count uint32[S]) like KvSketch.topk_all."""
        return self.keys[:, :k].copy(), self.est[:, :k].copy(), np.minimum(self.cnt, k).astype(np.uint32)


def kv_port(service_id, key_hash, num_services: int, width: int, depth: int = 4, candidates: int = 64, seed: int = 0,
            threads: int = 1) -> KvPortResult:
    """oracle/zk_kv_port.c: one batch into a fresh sketch, multithreaded (C4's checker on large
    prefixes and its CPU baseline). Same integers as KvOracle after one accumulate."""
    import ctypes as C

    from .oracle import lib

    svc = np.ascontiguousarray(service_id, dtype=np.uint32)
    keys = np.ascontiguousarray(np.asarray(key_hash).view(np.uint64) if np.asarray(key_hash).dtype == np.int64
                                else key_hash, dtype=np.uint64)
    S = num_services
    cm = np.zeros((S, depth, width), np.uint32)
    totals = np.zeros(S, np.uint64)
    ok = np.zeros((S, candidates), np.uint64)
    oe = np.zeros((S, candidates), np.uint32)
    cnt = np.zeros(S, np.uint32)
    dropped = np.zeros(1, np.uint64)
    secs = C.c_double()
    rc = lib().zkv_port(svc.ctypes.data, keys.ctypes.data, len(svc), S, width, depth, candidates, seed, threads,
                        cm.ctypes.data, totals.ctypes.data, ok.ctypes.data, oe.ctypes.data, cnt.ctypes.data,
                        dropped.ctypes.data, C.byref(secs))
    if rc != 0:
        raise ValueError("zkv_port: bad arguments or out of memory")
    return KvPortResult(cm, totals, ok, oe, cnt, int(dropped[0]), secs.value, threads)
