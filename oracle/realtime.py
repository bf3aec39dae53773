"""CPU restatement of the realtime span sketches (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module, as the
checker. It restates, in numpy, what include/zksketch.h (zk_rt_*) promises:

* the items: one per merged span -- fragments grouped by (traceId, spanId), Span.mergeSpan
  (zipkin-common/.../common/Span.scala:148-169) -- that passes Span.isValid (:236-240, every core
  annotation at most once) and has Span.serviceName (:125-131, server side first), carrying
  (service, traceId, duration = last - first annotation, :228-230);
* HyperLogLog per service: h = mix64(traceId ^ seed ^ SALT) (splitmix64 finalizer; the salt
  decorrelates it from the traceId shard hash, which is splitmix64 too), register index =
  top p bits, value = leading zeros of h << p, plus one (64 - p + 1 when h << p == 0); register =
  max over items; estimate alpha_m m^2 / sum 2^-M with linear counting m ln(m/V) when the raw
  estimate is <= 2.5 m and V registers are 0 (Flajolet, Fusy, Gandouet, Meunier 2007);
* the log-linear duration histogram with m mantissa bits: bin(d) = d below 2^m, else
  ((e - m + 1) << m) | top m mantissa bits of d, e = floor(log2 d).

The reference implements none of this (RealtimeAggregates.scala:26-38 is an interface;
QueryService.scala:416-430 answers "Not Implemented"): parity of the product against this file
is exact (same registers, same counts, same estimates); the sketches' contract against exact
answers (`exact_distinct`, `exact_quantile`) is the stated error bound -- "parity unpinned"
against the reference, which computes nothing here.
"""
from __future__ import annotations

import math

import numpy as np

from .kv import mix64

PAY_SHIFT_RHO = 40
MAX_DURATION = 1 << 40
SALT = 0xD6E8FEB86659FD93
F_HAS_ANNOTATIONS = 1 << 1
F_SVC_CLIENT = 1 << 2
F_SVC_SERVER = 1 << 3


def nbins(m: int) -> int:
    return (41 - m) << m


def bins_of(d: np.ndarray, m: int) -> np.ndarray:
    d = np.asarray(d, dtype=np.uint64)
    out = d.astype(np.int64)
    big = d >= np.uint64(1 << m)
    if big.any():
        db = d[big]
        e = np.frexp(db.astype(np.float64))[1].astype(np.int64) - 1  # exact: d < 2^40 < 2^53
        mant = (db >> (e - m).astype(np.uint64)) & np.uint64((1 << m) - 1)
        out[big] = ((e - m + 1) << m) | mant.astype(np.int64)
    return out


def bin_bounds(b: int, m: int) -> tuple[int, int]:
    if b < (1 << m):
        return b, b
    g, mant = b >> m, b & ((1 << m) - 1)
    e = g + m - 1
    lo = ((1 << m) | mant) << (e - m)
    return lo, lo + (1 << (e - m)) - 1


def hll_fields(trace_id: np.ndarray, p: int, seed: int):
    h = mix64(np.asarray(trace_id, dtype=np.uint64) ^ np.uint64(seed) ^ np.uint64(SALT))
    idx = (h >> np.uint64(64 - p)).astype(np.int64)
    w = (h << np.uint64(p)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    # leading zeros of w (64-bit) + 1; w == 0 -> 64 - p + 1
    rho = np.full(len(w), 64 - p + 1, dtype=np.int64)
    nz = w != 0
    if nz.any():
        wf = w[nz]
        hi = (wf >> np.uint64(32)).astype(np.uint64)
        lo = (wf & np.uint64(0xFFFFFFFF)).astype(np.uint64)
        # exact bit length via frexp on 32-bit halves
        bl_hi = np.frexp(hi.astype(np.float64))[1].astype(np.int64)
        bl_lo = np.frexp(lo.astype(np.float64))[1].astype(np.int64)
        bitlen = np.where(hi != 0, 32 + bl_hi, bl_lo)
        rho[nz] = 64 - bitlen + 1
    return idx, rho


def hll_estimate(regs: np.ndarray, p: int) -> float:
    """Same arithmetic as zk_rt_distinct_traces (exact integer sum, one rounding)."""
    m = 1 << p
    z = sum(1 << (64 - int(r)) for r in regs)
    zeros = int(np.count_nonzero(regs == 0))
    Z = float(z) / float(1 << 64)
    mf = float(m)
    if m == 16:
        alpha = 0.673
    elif m == 32:
        alpha = 0.697
    elif m == 64:
        alpha = 0.709
    else:
        alpha = 0.7213 / (1.0 + 1.079 / mf)
    e = alpha * mf * mf / Z
    if e <= 2.5 * mf and zeros > 0:
        e = mf * math.log(mf / float(zeros))
    return e


def nearest_rank(q: float, n: int) -> int:
    r = math.ceil(q * float(n))
    return min(max(r, 1), n)


class RtOracle:
    def __init__(self, num_services: int, p: int = 14, m: int = 7, seed: int = 0):
        self.S, self.p, self.m, self.seed = num_services, p, m, seed
        self.regs = np.zeros((num_services, 1 << p), np.uint8)
        self.hist = np.zeros((num_services, nbins(m)), np.uint64)
        self.dropped_service = 0
        self.dropped_duration = 0

    def accumulate_merged(self, service_id, trace_id, duration) -> None:
        svc = np.asarray(service_id, dtype=np.int64)
        tid = np.asarray(trace_id).view(np.uint64) if np.asarray(trace_id).dtype == np.int64 else \
            np.asarray(trace_id, dtype=np.uint64)
        dur = np.asarray(duration, dtype=np.int64)
        bad_s = (svc < 0) | (svc >= self.S)
        bad_d = ~bad_s & ((dur < 0) | (dur >= MAX_DURATION))
        self.dropped_service += int(bad_s.sum())
        self.dropped_duration += int(bad_d.sum())
        ok = ~(bad_s | bad_d)
        svc, tid, dur = svc[ok], tid[ok], dur[ok]
        idx, rho = hll_fields(tid, self.p, self.seed)
        np.maximum.at(self.regs, (svc, idx), rho.astype(np.uint8))
        np.add.at(self.hist, (svc, bins_of(dur, self.m)), np.uint64(1))

    def distinct(self) -> np.ndarray:
        return np.array([hll_estimate(self.regs[s], self.p) for s in range(self.S)])

    def quantile_bins(self, s: int, qs):
        h = self.hist[s]
        n = int(h.sum())
        out = []
        cum = np.cumsum(h)
        for q in qs:
            if n == 0:
                out.append((0, 0))
                continue
            r = nearest_rank(q, n)
            b = int(np.searchsorted(cum, r, side="left"))
            out.append(bin_bounds(b, self.m))
        return out, n


def merged_span_items(cols, num_services: int):
    """(service, traceId, duration, dropped_duration) of every merged, valid span with a service
    and annotations, from columnar fragments (Span.mergeSpan / isValid / serviceName / duration)."""
    tid = np.asarray(cols.trace_id, dtype=np.uint64)
    sid = np.asarray(cols.span_id, dtype=np.uint64)
    flags = np.asarray(cols.flags, dtype=np.uint32)
    svc = np.asarray(cols.service_id, dtype=np.uint32)
    first = np.asarray(cols.first_ts, dtype=np.int64)
    last = np.asarray(cols.last_ts, dtype=np.int64)
    n = len(tid)
    if n == 0:
        z = np.zeros(0, np.int64)
        return z, z.astype(np.uint64), z, 0
    order = np.lexsort((sid, tid))
    tid_s, sid_s = tid[order], sid[order]
    start = np.r_[True, (tid_s[1:] != tid_s[:-1]) | (sid_s[1:] != sid_s[:-1])]
    gid = np.cumsum(start) - 1
    G = int(gid[-1]) + 1
    f = flags[order]
    ha = (f & F_HAS_ANNOTATIONS) != 0
    fmin = np.full(G, np.iinfo(np.int64).max, np.int64)
    lmax = np.full(G, np.iinfo(np.int64).min, np.int64)
    np.minimum.at(fmin, gid[ha], first[order][ha])
    np.maximum.at(lmax, gid[ha], last[order][ha])
    # service key: (kind << 30) | id, server (0) before client (1), min over fragments
    kind = np.where(f & F_SVC_SERVER, 0, np.where(f & F_SVC_CLIENT, 1, 2)).astype(np.int64)
    s_ = svc[order].astype(np.int64)
    has = (kind < 2) & (s_ < num_services)
    key = np.full(G, 1 << 62, np.int64)
    np.minimum.at(key, gid[has], (kind[has] << 30) | s_[has])
    counts = np.zeros((G, 4), np.int64)
    for c, sh in enumerate((8, 10, 12, 14)):
        np.add.at(counts[:, c], gid, ((f >> sh) & 3).astype(np.int64))
    valid = (counts <= 1).all(axis=1)
    keep = valid & (key != (1 << 62)) & (fmin != np.iinfo(np.int64).max)
    d = lmax - fmin
    bad = (d < 0) | (d >= MAX_DURATION)  # the device takes last - first as unsigned
    dropped = int((keep & bad).sum())
    keep &= ~bad
    gtid = tid_s[start]
    return (key[keep] & ((1 << 30) - 1)), gtid[keep], d[keep], dropped


def exact_distinct(service_id, trace_id, num_services: int) -> np.ndarray:
    svc = np.asarray(service_id, dtype=np.int64)
    tid = np.asarray(trace_id, dtype=np.uint64)
    out = np.zeros(num_services, np.int64)
    if len(svc) == 0:
        return out
    pairs = np.unique(np.stack([svc.astype(np.uint64), tid], 1), axis=0)
    np.add.at(out, pairs[:, 0].astype(np.int64), 1)
    return out


def exact_quantile(durations: np.ndarray, q: float) -> int:
    d = np.sort(np.asarray(durations, dtype=np.int64))
    return int(d[nearest_rank(q, len(d)) - 1])


# ---- t-digest over the histogram (zk_rt_tdigest, zipkin_amd/csrc/zk_rt_api.cpp) --------------------
# Restates the library's build: Dunning's merging t-digest with the k1 scale function
# k(q) = delta / (2 pi) asin(2q - 1) (T. Dunning, O. Ertl, "Computing extremely accurate quantiles
# using t-digests", 2019; the published algorithm, no library source), fed with the histogram's
# nonzero bins in ascending order as (midpoint, count) points; a bin is never split.
def tdigest(hist_row, m: int, delta: float):
    h = np.asarray(hist_row, dtype=np.uint64)
    N = int(h.sum())
    if N == 0:
        return [], 0, 0, 0
    def k_of(q):
        return delta / (2 * math.pi) * math.asin(2 * q - 1)
    def q_of(k):
        x = 2 * math.pi * k / delta
        return 1.0 if x >= math.pi / 2 else (math.sin(x) + 1) / 2
    cent = []
    first = True
    before = cw = cs = qlim = 0.0
    vmin = vmax = 0
    for b in np.flatnonzero(h):
        lo, hi = bin_bounds(int(b), m)
        if first:
            vmin = lo
        vmax = hi
        w, x = float(h[b]), 0.5 * (float(lo) + float(hi))
        if not first and (before + cw + w) / N <= qlim:
            cw += w
            cs += w * x
            continue
        if not first:
            cent.append((cs / cw, cw))
            before += cw
        first = False
        cw, cs = w, w * x
        qlim = q_of(k_of(before / N) + 1.0)
    cent.append((cs / cw, cw))
    return cent, vmin, vmax, N


def tdigest_quantile(cent, vmin: int, vmax: int, N: int, q: float) -> float:
    if not cent or N == 0:
        return 0.0
    if len(cent) == 1:
        return cent[0][0]
    idx = q * N
    if idx <= cent[0][1] / 2:
        t = idx / (cent[0][1] / 2) if cent[0][1] > 0 else 0.0
        return vmin + t * (cent[0][0] - vmin)
    cum = 0.0
    for i in range(len(cent) - 1):
        a = cum + cent[i][1] / 2
        b = cum + cent[i][1] + cent[i + 1][1] / 2
        if idx <= b:
            t = (idx - a) / (b - a) if b > a else 0.0
            return cent[i][0] + t * (cent[i + 1][0] - cent[i][0])
        cum += cent[i][1]
    mean, w = cent[-1]
    a = N - w / 2
    t = (idx - a) / (w / 2) if w > 0 else 0.0
    return mean + min(t, 1.0) * (vmax - mean)


class RtPortResult:
    def __init__(self, regs, hist, dropped, seconds, threads):
        self.regs, self.hist, self.seconds, self.threads = regs, hist, seconds, threads
        self.dropped_service, self.dropped_duration = int(dropped[0]), int(dropped[1])
        self.p = int(regs.shape[1]).bit_length() - 1

    def distinct(self) -> np.ndarray:
        return np.array([hll_estimate(self.regs[s], self.p) for s in range(self.regs.shape[0])])


def rt_port(cols, num_services: int, p: int = 14, m: int = 7, seed: int = 0, threads: int = 1) -> RtPortResult:
    """oracle/zk_rt_port.c: one TRACE-CLUSTERED batch into fresh sketches, multithreaded (C5's
    checker on large prefixes and its CPU baseline). Same registers and bins as
    RtOracle.accumulate_merged(*merged_span_items(cols)) (tests/test_realtime.py)."""
    import ctypes as C

    from .oracle import lib

    arrs = [np.ascontiguousarray(cols.trace_id, np.uint64), np.ascontiguousarray(cols.span_id, np.uint64),
            np.ascontiguousarray(cols.first_ts, np.int64), np.ascontiguousarray(cols.last_ts, np.int64),
            np.ascontiguousarray(cols.service_id, np.uint32), np.ascontiguousarray(cols.flags, np.uint32)]
    S = num_services
    regs = np.zeros((S, 1 << p), np.uint8)
    hist = np.zeros((S, nbins(m)), np.uint64)
    dropped = np.zeros(2, np.uint64)
    secs = C.c_double()
    rc = lib().zkr_port(*[a.ctypes.data for a in arrs], len(arrs[0]), S, p, m, seed, threads, regs.ctypes.data,
                        hist.ctypes.data, dropped.ctypes.data, C.byref(secs))
    if rc != 0:
        raise ValueError("zkr_port: bad arguments or out of memory")
    return RtPortResult(regs, hist, dropped, secs.value, threads)


# ---- the realtime link store (zk_rl_*, RealtimeAggregates) --------------------------------------
F_HAS_PARENT = 1 << 0


def joined_links(cols, num_services: int):
    """Every join row of the dependency job, before its group.sum: (parent service, child service,
    child duration, traceId) per joined child span -- ZipkinAggregateJob.scala:21-37 on columnar
    fragments: mergeSpan over (traceId, spanId) (Span.scala:148-169; parentId = the min over the
    fragments that carry one, the deterministic rule zk_oracle.c uses), isValid (:236-240), the join
    on (parentId, traceId) against a valid merged parent, both serviceNames (:125-131, server side
    first), duration = last - first annotation (:228-230) below 2^40 us. Returns four arrays in
    (parent, child, duration, traceId) order."""
    tid = np.asarray(cols.trace_id, dtype=np.uint64)
    sid = np.asarray(cols.span_id, dtype=np.uint64)
    pid = np.asarray(cols.parent_id, dtype=np.uint64)
    flags = np.asarray(cols.flags, dtype=np.uint32)
    svc = np.asarray(cols.service_id, dtype=np.uint32)
    first = np.asarray(cols.first_ts, dtype=np.int64)
    last = np.asarray(cols.last_ts, dtype=np.int64)
    empty = (np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.uint64))
    if len(tid) == 0:
        return empty
    order = np.lexsort((sid, tid))
    tid_s, sid_s, f = tid[order], sid[order], flags[order]
    start = np.r_[True, (tid_s[1:] != tid_s[:-1]) | (sid_s[1:] != sid_s[:-1])]
    gid = np.cumsum(start) - 1
    G = int(gid[-1]) + 1
    ha = (f & F_HAS_ANNOTATIONS) != 0
    fmin = np.full(G, np.iinfo(np.int64).max, np.int64)
    lmax = np.full(G, np.iinfo(np.int64).min, np.int64)
    np.minimum.at(fmin, gid[ha], first[order][ha])
    np.maximum.at(lmax, gid[ha], last[order][ha])
    kind = np.where(f & F_SVC_SERVER, 0, np.where(f & F_SVC_CLIENT, 1, 2)).astype(np.int64)
    s_ = svc[order].astype(np.int64)
    has = (kind < 2) & (s_ < num_services)
    key = np.full(G, 1 << 62, np.int64)
    np.minimum.at(key, gid[has], (kind[has] << 30) | s_[has])
    counts = np.zeros((G, 4), np.int64)
    for c, sh in enumerate((8, 10, 12, 14)):
        np.add.at(counts[:, c], gid, ((f >> sh) & 3).astype(np.int64))
    valid = (counts <= 1).all(axis=1)
    hp = (f & F_HAS_PARENT) != 0
    gpar = np.full(G, np.iinfo(np.uint64).max, np.uint64)
    np.minimum.at(gpar, gid[hp], pid[order][hp])
    has_par = np.zeros(G, bool)
    has_par[gid[hp]] = True
    gtid, gsid = tid_s[start], sid_s[start]
    # the parent: the merged span (traceId, parentId), valid
    child = np.flatnonzero(valid & has_par)
    lo = np.searchsorted(gtid, gtid[child], side="left")
    hi = np.searchsorted(gtid, gtid[child], side="right")
    par = np.full(len(child), -1, np.int64)
    for i, (a, b) in enumerate(zip(lo, hi)):  # (a trace's groups are contiguous and spanId-sorted)
        j = a + int(np.searchsorted(gsid[a:b], gpar[child[i]]))
        if j < b and gsid[j] == gpar[child[i]] and valid[j]:
            par[i] = j
    ok = par >= 0
    child, par = child[ok], par[ok]
    none = 1 << 62
    ok = (key[child] != none) & (key[par] != none)
    child, par = child[ok], par[ok]
    d = lmax[child] - fmin[child]
    ok = (fmin[child] != np.iinfo(np.int64).max) & (d >= 0) & (d < MAX_DURATION)
    child, par, d = child[ok], par[ok], d[ok]
    mask = (1 << 30) - 1
    return key[par] & mask, key[child] & mask, d, gtid[child]


def server_links(links, server: int):
    """The rows of `server` (the child side), ordered by (parent, duration, traceId): what
    zk_rl_server_links returns."""
    p, c, d, t = links
    sel = np.flatnonzero(c == server)
    o = np.lexsort((t[sel], d[sel], p[sel]))
    return p[sel][o], d[sel][o], t[sel][o]
