// zk_store.cpp — the Aggregates store surface (include/zkstore.h): host-side, thread-safe.
//
// What the reference's Aggregates implementations persist and return
// (zipkin-common/.../storage/Aggregates.scala:26-37):
//   * AnormAggregates (zipkin-anormdb/.../storage/anormdb/AnormAggregates.scala:52-109): one row per
//     stored Dependencies (start_ts, end_ts) plus its links; getDependencies returns the links of
//     every row CONTAINED in [start, end] (start_ts >= start AND end_ts <= end), newest row first,
//     as Dependencies(start, end, links) with the defaults start = now - 1 day, end = now.
//   * CassandraAggregates (zipkin-cassandra/.../storage/cassandra/CassandraAggregates.scala):
//     storeDependencies writes row key startTime.floor(1.day) in us and store() clobbers the row
//     (removeRow, then column index 0 -> the record, :111-116,122-136); getDependencies walks every
//     row and keeps a column unless its NAME -- the index 0, not a time -- exceeds a given bound in
//     us (:58-61), then Monoid-sums the records (:69-71).
//   * HBaseAggregates (zipkin-hbase/.../storage/hbase/HBaseAggregates.scala): row key
//     Long.MaxValue - startTime.inMilliseconds (:56-60, a later put of the same key replaces the
//     record); getDependencies scans [MaxValue - start ms (0 without a start), MaxValue - end ms)
//     in row-key byte order (:39-53) -- records with end < start ms <= start bound, newest first --
//     and Monoid-sums them.
//   Monoid.sum is reduceLeftOption(plus) over the rows in scan order (Dependencies.scala:65-82;
//   links merged per (parent, child) by DependencyLink.sg = algebird MomentsGroup.plus, :38-43),
//   the monoid zero when nothing matches.
//   * top annotation lists (Anorm: stubs, AnormAggregates.scala:111-137): a per-service list replaced wholesale by store* and read back in
//     list order (CassandraAggregates.scala:79-108,119-136). HBase (HBaseAggregates.scala:62-110)
//     writes both kinds into the top-annotation family, so getTopKeyValueAnnotations finds nothing;
//     getTopAnnotations returns the newest list stored under the first service id >= the asked one
//     (its scan has a start row and no stop row).
// Dictionary ids stand in for the strings (the host owns the dictionaries, as for zkagg.h).
#include <math.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "zk_guard.h"
#include "zkstore.h"

namespace {

constexpr int64_t kDayUs = 86400LL * 1000000LL;

struct StoredDeps {
    int64_t start, end;
    std::vector<zk_dep_link> links;
};

// algebird-core 0.8.1 Moments.getCombinedMean (STABILITY_CONSTANT = 0.1)
double combined_mean(int64_t n, double an, int64_t k, double ak) {
    if (n < k) return combined_mean(k, ak, n, an);
    const int64_t nc = n + k;
    if (nc == 0) return 0.0;
    if (nc == n) return an;
    const double scaling = (double)k / (double)nc;
    if (scaling < 0.1) return an + (ak - an) * scaling;
    return ((double)n * an + (double)k * ak) / (double)nc;
}

// algebird-core 0.8.1 MomentsGroup.plus, in its own evaluation order (math.pow for the powers)
zk_moments moments_plus(const zk_moments& a, const zk_moments& b) {
    const double delta = b.m1 - a.m1;
    const int64_t nc = a.m0 + b.m0;
    zk_moments r{0, 0.0, 0.0, 0.0, 0.0};
    if (nc == 0) return r;
    const double na = (double)a.m0, nb = (double)b.m0, n = (double)nc;
    r.m0 = nc;
    r.m1 = combined_mean(a.m0, a.m1, b.m0, b.m1);
    r.m2 = a.m2 + b.m2 + pow(delta, 2) * na * nb / n;
    r.m3 = a.m3 + b.m3 + pow(delta, 3) * na * nb * (double)(a.m0 - b.m0) / pow(n, 2) +
           3 * delta * (na * b.m2 - nb * a.m2) / n;
    r.m4 = a.m4 + b.m4 +
           pow(delta, 4) * na * nb * (pow(na, 2) - na * nb + pow(nb, 2)) / pow(n, 3) +
           6 * pow(delta, 2) * (pow(na, 2) * b.m2 + pow(nb, 2) * a.m2) / pow(n, 2) +
           4 * delta * (na * b.m3 - nb * a.m3) / n;
    return r;
}

}  // namespace

struct zk_store {
    std::mutex mu;
    uint32_t mode = ZK_STORE_ANORM;
    std::vector<StoredDeps> rows;            // Anorm: insertion order (dlid)
    std::map<uint64_t, StoredDeps> keyed;    // Cassandra / HBase: row key (unsigned = byte order)
    std::map<uint32_t, std::vector<uint64_t>> top[2];
    std::string err;
};

namespace {

zk_status sfail(zk_store* s, zk_status st, const char* msg) {
    s->err = msg;
    return st;
}

// 8-byte big-endian row keys compare as unsigned integers (Cassandra row order under a byte-ordered
// partitioner, HBase's lexicographic row order); Long arithmetic wraps like the JVM's
uint64_t cassandra_key(int64_t start_us) { return (uint64_t)((start_us / kDayUs) * kDayUs); }  // Time.floor: Long division
uint64_t hbase_key_ms(int64_t ms) { return (uint64_t)INT64_MAX - (uint64_t)ms; }

// Monoid.sum over records in order: reduceLeftOption(Dependencies.plus), zero if none. A single
// record comes back as stored; from two on, every operand goes through `links.map(k -> link).toMap`
// (the last link of a duplicated key wins) and shared keys combine as sg.plus(r, l)
// (Dependencies.scala:68-79). MomentsGroup.plus is bitwise symmetric, so only the left fold over
// records fixes the rounding.
void monoid_sum(const std::vector<const StoredDeps*>& hit, std::vector<zk_dep_link>* res, int64_t* rs,
                int64_t* re) {
    *rs = ZK_TIME_TOP;
    *re = ZK_TIME_BOTTOM;
    if (hit.size() == 1) {
        *rs = hit[0]->start;
        *re = hit[0]->end;
        *res = hit[0]->links;
        return;
    }
    std::map<std::pair<uint32_t, uint32_t>, zk_moments> acc;
    for (size_t r = 0; r < hit.size(); ++r) {
        const StoredDeps& d = *hit[r];
        *rs = std::min(*rs, d.start);
        *re = std::max(*re, d.end);
        std::map<std::pair<uint32_t, uint32_t>, zk_moments> m;
        for (const zk_dep_link& l : d.links) m[std::make_pair(l.parent, l.child)] = l.moments;
        if (r == 0) {
            acc = std::move(m);
            continue;
        }
        for (const auto& kv : m) {
            auto it = acc.find(kv.first);
            if (it == acc.end())
                acc.emplace(kv.first, kv.second);
            else
                it->second = moments_plus(kv.second, it->second);
        }
    }
    for (const auto& kv : acc) res->push_back(zk_dep_link{kv.first.first, kv.first.second, kv.second});
}

}  // namespace

extern "C" {

zk_status zk_store_create(uint32_t mode, zk_store** out) {
    ZK_GUARD_BEGIN
    if (!out) return ZK_ERR_INVALID_ARG;
    *out = nullptr;
    if (mode != ZK_STORE_ANORM && mode != ZK_STORE_CASSANDRA && mode != ZK_STORE_HBASE) return ZK_ERR_INVALID_ARG;
    zk_store* s = new zk_store();
    s->mode = mode;
    *out = s;
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_store_destroy(zk_store* s) {
    ZK_GUARD_BEGIN
    if (!s) return ZK_ERR_INVALID_ARG;
    delete s;
    return ZK_OK;
    ZK_GUARD_END
}

const char* zk_store_last_error(const zk_store* s) { return s ? s->err.c_str() : "null store"; }

zk_status zk_store_put_dependencies(zk_store* s, int64_t start_us, int64_t end_us, const zk_dep_link* links,
                                    uint64_t n) {
    ZK_GUARD_BEGIN
    if (!s) return ZK_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(s->mu);
    if (n && !links) return sfail(s, ZK_ERR_INVALID_ARG, "null links");
    StoredDeps d;
    d.start = start_us;
    d.end = end_us;
    d.links.assign(links, links + n);
    if (s->mode == ZK_STORE_CASSANDRA)
        s->keyed[cassandra_key(start_us)] = std::move(d);  // removeRow + insert (:111-116,122-136)
    else if (s->mode == ZK_STORE_HBASE)
        s->keyed[hbase_key_ms(start_us / 1000)] = std::move(d);  // Put replaces the row's cell (:55-60)
    else
        s->rows.push_back(std::move(d));
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_store_get_dependencies(zk_store* s, const int64_t* start_us, const int64_t* end_us, int64_t now_us,
                                    zk_dep_link* out, uint64_t cap, uint64_t* n_links, int64_t* out_start,
                                    int64_t* out_end) {
    ZK_GUARD_BEGIN
    if (!s || !n_links) return ZK_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(s->mu);
    std::vector<zk_dep_link> res;
    int64_t rs, re;
    if (s->mode == ZK_STORE_CASSANDRA) {
        // every row, column 0 kept unless a given bound is below 0 us (CassandraAggregates.scala:58-61)
        std::vector<const StoredDeps*> hit;
        const bool keep = !(end_us && 0 > *end_us) && !(start_us && 0 > *start_us);
        if (keep)
            for (const auto& kv : s->keyed) hit.push_back(&kv.second);
        monoid_sum(hit, &res, &rs, &re);
    } else if (s->mode == ZK_STORE_HBASE) {
        // scan [startRow, stopRow) in row-key order (HBaseAggregates.scala:41-43); a start row past
        // the stop row scans nothing; startRow == stopRow is a get-scan (HBase's Scan.isGetScan:
        // the stop row is inclusive), which returns the record stored under that one key
        const uint64_t lo_key = hbase_key_ms(start_us ? *start_us / 1000 : INT64_MAX);
        const bool has_stop = end_us != nullptr;
        const uint64_t hi_key = has_stop ? hbase_key_ms(*end_us / 1000) : 0;
        std::vector<const StoredDeps*> hit;
        if (has_stop && lo_key == hi_key) {
            const auto it = s->keyed.find(lo_key);
            if (it != s->keyed.end()) hit.push_back(&it->second);
        } else if (!has_stop || lo_key < hi_key) {
            for (auto it = s->keyed.lower_bound(lo_key); it != s->keyed.end(); ++it) {
                if (has_stop && it->first >= hi_key) break;
                hit.push_back(&it->second);
            }
        }
        monoid_sum(hit, &res, &rs, &re);
    } else {
        const int64_t lo = start_us ? *start_us : now_us - kDayUs;  // AnormAggregates.scala:53-54
        const int64_t hi = end_us ? *end_us : now_us;
        // WHERE start_ts >= {startTs} AND end_ts <= {endTs} ORDER BY dlid DESC (:56-64)
        for (size_t i = s->rows.size(); i-- > 0;) {
            const StoredDeps& d = s->rows[i];
            if (d.start >= lo && d.end <= hi) res.insert(res.end(), d.links.begin(), d.links.end());
        }
        rs = lo;
        re = hi;
    }
    *n_links = res.size();
    if (out_start) *out_start = rs;
    if (out_end) *out_end = re;
    if (!out) return ZK_OK;
    if (cap < res.size()) return sfail(s, ZK_ERR_CAPACITY, "output capacity smaller than the result");
    if (!res.empty()) memcpy(out, res.data(), res.size() * sizeof(zk_dep_link));
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_store_count(zk_store* s, uint64_t* records) {
    ZK_GUARD_BEGIN
    if (!s || !records) return ZK_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(s->mu);
    *records = s->mode == ZK_STORE_ANORM ? s->rows.size() : s->keyed.size();
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_store_watermark(zk_store* s, int64_t* end_us) {
    ZK_GUARD_BEGIN
    if (!s || !end_us) return ZK_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(s->mu);
    int64_t w = 0;
    bool any = false;
    for (const StoredDeps& d : s->rows) {
        w = any ? std::max(w, d.end) : d.end;
        any = true;
    }
    for (const auto& kv : s->keyed) {
        w = any ? std::max(w, kv.second.end) : kv.second.end;
        any = true;
    }
    *end_us = any ? w : 0;
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_store_put_top(zk_store* s, uint32_t kind, uint32_t service, const uint64_t* ids, uint64_t n) {
    ZK_GUARD_BEGIN
    if (!s) return ZK_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(s->mu);
    if (kind > ZK_TOP_KV_ANNOTATIONS) return sfail(s, ZK_ERR_INVALID_ARG, "unknown top-annotation kind");
    if (n && !ids) return sfail(s, ZK_ERR_INVALID_ARG, "null ids");
    // store(): removeRow(key) then insert column i -> value i (CassandraAggregates.scala:122-136).
    // HBase puts both kinds into the top-annotation family, the newest put read first
    // (HBaseAggregates.scala:104-110): one list per service, whichever kind stored it last.
    // Anorm's top-annotation methods are stubs (AnormAggregates.scala:111-137): nothing is kept.
    if (s->mode == ZK_STORE_ANORM) return ZK_OK;
    s->top[s->mode == ZK_STORE_HBASE ? 0 : kind][service].assign(ids, ids + n);
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_store_get_top(zk_store* s, uint32_t kind, uint32_t service, uint64_t* ids, uint64_t cap, uint64_t* n) {
    ZK_GUARD_BEGIN
    if (!s || !n) return ZK_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> g(s->mu);
    if (kind > ZK_TOP_KV_ANNOTATIONS) return sfail(s, ZK_ERR_INVALID_ARG, "unknown top-annotation kind");
    auto it = s->top[kind].find(service);
    if (s->mode == ZK_STORE_HBASE) {
        // the key-value family is never written; the annotation scan starts at (service id, 0) with
        // no stop row and takes the first row, which belongs to the next stored service id when
        // this one has none (HBaseAggregates.scala:70-94)
        it = kind == ZK_TOP_KV_ANNOTATIONS ? s->top[0].end() : s->top[0].lower_bound(service);
        if (kind == ZK_TOP_KV_ANNOTATIONS) {
            *n = 0;
            return ZK_OK;
        }
    }
    const auto& tk = s->top[s->mode == ZK_STORE_HBASE ? 0 : kind];
    const uint64_t cnt = it == tk.end() ? 0 : it->second.size();
    *n = cnt;
    if (!ids || cnt == 0) return ZK_OK;
    if (cap < cnt) return sfail(s, ZK_ERR_CAPACITY, "output capacity smaller than the list");
    memcpy(ids, it->second.data(), cnt * sizeof(uint64_t));
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_moments_plus(const zk_moments* a, const zk_moments* b, zk_moments* out) {
    ZK_GUARD_BEGIN
    if (!a || !b || !out) return ZK_ERR_INVALID_ARG;
    *out = moments_plus(*a, *b);
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_link_table_compact(const zk_link_table* t, uint32_t S, zk_dep_link* out, uint64_t cap, uint64_t* n) {
    ZK_GUARD_BEGIN
    if (!t || !n || !t->m0 || !t->m1 || !t->m2 || !t->m3 || !t->m4 || !t->present || t->device_ptrs)
        return ZK_ERR_INVALID_ARG;
    const uint64_t cells = (uint64_t)S * S;
    uint64_t k = 0;
    for (uint64_t c = 0; c < cells; ++c) {
        if (!t->present[c]) continue;
        if (out) {
            if (k >= cap) return ZK_ERR_CAPACITY;
            out[k] = zk_dep_link{(uint32_t)(c / S), (uint32_t)(c % S),
                                 zk_moments{(int64_t)t->m0[c], t->m1[c], t->m2[c], t->m3[c], t->m4[c]}};
        }
        ++k;
    }
    *n = k;
    return ZK_OK;
    ZK_GUARD_END
}

}  // extern "C"
