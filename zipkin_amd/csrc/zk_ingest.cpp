// zk_ingest.cpp — stored span fragments -> 48-B columnar records (include/zkingest.h).
//
// One pass per fragment: [raw Snappy block ->] TBinaryProtocol Span (zipkinCore.thrift:27-58) ->
// the reference's thrift validation (thrift.scala:36-121) -> the record of SURVEY Appendix A.1,
// plus the span indexer's key-value / annotation items (CassieSpanStore.scala:214-242).
// Every read is bounds-checked: corrupt input is an error, never a crash.
#include <string.h>

#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "zk_guard.h"
#include "zkingest.h"

namespace {

const char kUnknownService[] = "Unknown service name";  // Endpoint.UnknownServiceName

// ---- raw Snappy block (the format iq80 Snappy.compress writes, SnappyCodec.scala:34-41) -------
bool snappy_len(const uint8_t* in, uint64_t n, uint64_t* len, uint64_t* hdr) {
    uint64_t v = 0;
    for (uint64_t i = 0; i < n && i < 5; ++i) {
        v |= (uint64_t)(in[i] & 0x7F) << (7 * i);
        if (!(in[i] & 0x80)) {
            *len = v;
            *hdr = i + 1;
            return v <= 0xFFFFFFFFull;
        }
    }
    return false;
}

// the announced length is checked against the fragment cap and the format's expansion bound
// before anything is allocated (the device decoder applies the same rule)
bool snappy_len_ok(uint64_t len, uint64_t n, uint64_t hdr) {
    return len <= ZK_INGEST_MAX_FRAGMENT && len <= (n - hdr) * (uint64_t)ZK_SNAPPY_MAX_EXPANSION;
}

bool snappy_uncompress(const uint8_t* in, uint64_t n, std::vector<uint8_t>* out) {
    uint64_t len, hdr;
    if (!snappy_len(in, n, &len, &hdr) || !snappy_len_ok(len, n, hdr)) return false;
    out->resize(len);
    uint8_t* op = out->data();
    uint64_t o = 0;
    uint64_t i = hdr;
    while (i < n) {
        const uint8_t tag = in[i++];
        uint64_t l, off;
        switch (tag & 3) {
            case 0: {  // literal
                l = tag >> 2;
                if (l >= 60) {
                    const uint32_t nb = (uint32_t)l - 59;
                    if (i + nb > n) return false;
                    l = 0;
                    for (uint32_t k = 0; k < nb; ++k) l |= (uint64_t)in[i + k] << (8 * k);
                    i += nb;
                }
                l += 1;
                if (i + l > n || o + l > len) return false;
                memcpy(op + o, in + i, l);
                i += l;
                o += l;
                continue;
            }
            case 1:
                if (i + 1 > n) return false;
                l = ((tag >> 2) & 7) + 4;
                off = ((uint64_t)(tag >> 5) << 8) | in[i];
                i += 1;
                break;
            case 2:
                if (i + 2 > n) return false;
                l = (tag >> 2) + 1;
                off = (uint64_t)in[i] | ((uint64_t)in[i + 1] << 8);
                i += 2;
                break;
            default:
                if (i + 4 > n) return false;
                l = (tag >> 2) + 1;
                off = (uint64_t)in[i] | ((uint64_t)in[i + 1] << 8) | ((uint64_t)in[i + 2] << 16) |
                      ((uint64_t)in[i + 3] << 24);
                i += 4;
                break;
        }
        if (off == 0 || off > o || o + l > len) return false;
        for (uint64_t k = 0; k < l; ++k) op[o + k] = op[o - off + k];  // may overlap: bytewise
        o += l;
    }
    return o == len;
}

// ---- TBinaryProtocol ----------------------------------------------------------------------
enum TType : uint8_t {
    T_STOP = 0, T_BOOL = 2, T_BYTE = 3, T_DOUBLE = 4, T_I16 = 6, T_I32 = 8, T_I64 = 10, T_STRING = 11,
    T_STRUCT = 12, T_MAP = 13, T_SET = 14, T_LIST = 15
};

struct Rd {
    const uint8_t* p;
    const uint8_t* e;
    bool ok = true;
    bool need(uint64_t k) {
        if (!ok || (uint64_t)(e - p) < k) ok = false;
        return ok;
    }
    uint8_t u8() {
        if (!need(1)) return 0;
        return *p++;
    }
    int16_t i16() {
        if (!need(2)) return 0;
        const int16_t v = (int16_t)((p[0] << 8) | p[1]);
        p += 2;
        return v;
    }
    int32_t i32() {
        if (!need(4)) return 0;
        const uint32_t v = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
        p += 4;
        return (int32_t)v;
    }
    int64_t i64() {
        if (!need(8)) return 0;
        uint64_t v = 0;
        for (int k = 0; k < 8; ++k) v = (v << 8) | p[k];
        p += 8;
        return (int64_t)v;
    }
    bool str(const char** s, uint32_t* len) {
        const int32_t l = i32();
        if (!ok || l < 0 || !need((uint64_t)l)) return ok = false;
        *s = (const char*)p;
        *len = (uint32_t)l;
        p += l;
        return true;
    }
    void skip(uint8_t t, int depth = 0) {
        if (depth > 64) {
            ok = false;
            return;
        }
        switch (t) {
            case T_BOOL:
            case T_BYTE: u8(); break;
            case T_I16: i16(); break;
            case T_I32: i32(); break;
            case T_DOUBLE:
            case T_I64: i64(); break;
            case T_STRING: {
                const char* s;
                uint32_t l;
                str(&s, &l);
                break;
            }
            case T_STRUCT:
                for (;;) {
                    const uint8_t ft = u8();
                    if (!ok || ft == T_STOP) break;
                    i16();
                    skip(ft, depth + 1);
                }
                break;
            case T_MAP: {
                const uint8_t kt = u8(), vt = u8();
                const int32_t n = i32();
                if (n < 0) ok = false;
                for (int32_t k = 0; ok && k < n; ++k) {
                    skip(kt, depth + 1);
                    skip(vt, depth + 1);
                }
                break;
            }
            case T_SET:
            case T_LIST: {
                const uint8_t et = u8();
                const int32_t n = i32();
                if (n < 0) ok = false;
                for (int32_t k = 0; ok && k < n; ++k) skip(et, depth + 1);
                break;
            }
            default: ok = false;
        }
    }
};

struct Host {
    bool present = false;
    const char* svc = nullptr;  // null: absent field
    uint32_t svc_len = 0;
};
struct Ann {
    int64_t ts = 0;
    const char* value = nullptr;
    uint32_t value_len = 0;
    Host host;
};
struct BinAnn {
    const char* key = nullptr;
    uint32_t key_len = 0;
    Host host;
};
struct SpanT {
    int64_t trace_id = 0, id = 0, parent_id = 0;
    bool has_parent = false, has_name = false;
    std::vector<Ann> anns;
    std::vector<BinAnn> banns;
    void clear() {
        trace_id = id = parent_id = 0;
        has_parent = has_name = false;
        anns.clear();
        banns.clear();
    }
};

void read_endpoint(Rd& r, Host* h) {
    h->present = true;
    for (;;) {
        const uint8_t t = r.u8();
        if (!r.ok || t == T_STOP) return;
        const int16_t id = r.i16();
        if (id == 3 && t == T_STRING)
            r.str(&h->svc, &h->svc_len);
        else
            r.skip(t);
    }
}

void read_annotation(Rd& r, Ann* a) {
    for (;;) {
        const uint8_t t = r.u8();
        if (!r.ok || t == T_STOP) return;
        const int16_t id = r.i16();
        if (id == 1 && t == T_I64)
            a->ts = r.i64();
        else if (id == 2 && t == T_STRING)
            r.str(&a->value, &a->value_len);
        else if (id == 3 && t == T_STRUCT)
            read_endpoint(r, &a->host);
        else
            r.skip(t);
    }
}

void read_binary_annotation(Rd& r, BinAnn* b) {
    for (;;) {
        const uint8_t t = r.u8();
        if (!r.ok || t == T_STOP) return;
        const int16_t id = r.i16();
        if (id == 1 && t == T_STRING)
            r.str(&b->key, &b->key_len);
        else if (id == 4 && t == T_STRUCT)
            read_endpoint(r, &b->host);
        else
            r.skip(t);
    }
}

bool read_span(Rd& r, SpanT* s) {
    for (;;) {
        const uint8_t t = r.u8();
        if (!r.ok) return false;
        if (t == T_STOP) return true;
        const int16_t id = r.i16();
        if (id == 1 && t == T_I64) {
            s->trace_id = r.i64();
        } else if (id == 3 && t == T_STRING) {
            const char* nm;
            uint32_t l;
            s->has_name = r.str(&nm, &l);
        } else if (id == 4 && t == T_I64) {
            s->id = r.i64();
        } else if (id == 5 && t == T_I64) {
            s->parent_id = r.i64();
            s->has_parent = true;
        } else if ((id == 6 || id == 8) && t == T_LIST) {
            const uint8_t et = r.u8();
            const int32_t n = r.i32();
            if (!r.ok || n < 0 || et != T_STRUCT) {
                if (r.ok && n >= 0) {  // a list of something else: skip it
                    for (int32_t k = 0; r.ok && k < n; ++k) r.skip(et);
                    continue;
                }
                return false;
            }
            for (int32_t k = 0; r.ok && k < n; ++k) {
                if (id == 6) {
                    s->anns.emplace_back();
                    read_annotation(r, &s->anns.back());
                } else {
                    s->banns.emplace_back();
                    read_binary_annotation(r, &s->banns.back());
                }
            }
        } else {
            r.skip(t);
        }
        if (!r.ok) return false;
    }
}

bool is_core(const char* v, uint32_t l) {
    return v && l == 2 && ((v[0] == 'c' && (v[1] == 's' || v[1] == 'r')) || (v[0] == 's' && (v[1] == 'r' || v[1] == 's')));
}

// ---- TBinaryProtocol writer (the Dependencies record) -----------------------------------------
struct Wr {
    uint8_t* out;
    uint64_t cap, len = 0;
    void put(const void* p, uint64_t k) {
        if (out && len + k <= cap) memcpy(out + len, p, k);
        len += k;
    }
    void u8(uint8_t v) { put(&v, 1); }
    void be(uint64_t v, int bytes) {
        uint8_t b[8];
        for (int i = 0; i < bytes; ++i) b[i] = (uint8_t)(v >> (8 * (bytes - 1 - i)));
        put(b, bytes);
    }
    void field(uint8_t t, int16_t id) {
        u8(t);
        be((uint16_t)id, 2);
    }
    void i64(int16_t id, int64_t v) {
        field(T_I64, id);
        be((uint64_t)v, 8);
    }
    void dbl(int16_t id, double v) {
        uint64_t bits;
        memcpy(&bits, &v, 8);
        field(T_DOUBLE, id);
        be(bits, 8);
    }
    void str(int16_t id, const char* s, uint32_t l) {
        field(T_STRING, id);
        be(l, 4);
        put(s, l);
    }
};

double bits_double(int64_t v) {
    double d;
    memcpy(&d, &v, 8);
    return d;
}

uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

}  // namespace

// ---- phase 1 of zk_ingest_spans: one thread's range of fragments -------------------------------
constexpr uint32_t kIngestThreads = 16;          // decode threads (the GPU box gives a process 16 CPUs)
constexpr uint64_t kIngestMinPerThread = 2048;   // fragments per thread at least

struct Item {
    int32_t name;  // the host's service name: index into DecodeRange::names
    uint32_t str;  // the key / value string: index into DecodeRange::strs
    uint64_t hash;
};
struct Decoded {
    uint64_t index;  // fragment index in the batch
    uint64_t tid, sid, pid;
    int64_t first, last;
    uint32_t flags;
    int32_t svc_name;  // -1: no service
    uint32_t kv0, kv_n, ann0, ann_n;
};
struct DecodeRange {
    uint64_t lo = 0, hi = 0;
    std::vector<Decoded> recs;
    std::vector<Item> kv, ann;
    std::vector<std::string> names, strs;
    std::unordered_map<std::string, int32_t> name_ix;
    std::unordered_map<uint64_t, uint32_t> str_ix;
    uint64_t rejected = 0;
    uint64_t err_index = UINT64_MAX;  // first fragment that fails the batch (strict / bad offsets)
    zk_status err_status = ZK_OK;
    std::string err;

    int32_t name(const Host& h) {  // thrift.scala:36-43: null or "" -> Endpoint.UnknownServiceName
        std::string s = (h.svc && h.svc_len) ? std::string(h.svc, h.svc_len) : std::string(kUnknownService);
        auto it = name_ix.find(s);
        if (it != name_ix.end()) return it->second;
        const int32_t ix = (int32_t)names.size();
        name_ix.emplace(s, ix);
        names.push_back(std::move(s));
        return ix;
    }
    Item item(const Host& h, const char* s, uint32_t l) {
        const uint64_t hash = zk_hash_string(s, l);
        auto it = str_ix.find(hash);
        uint32_t ix;
        if (it != str_ix.end()) {
            ix = it->second;
        } else {
            ix = (uint32_t)strs.size();
            str_ix.emplace(hash, ix);
            strs.emplace_back(s ? s : "", s ? l : 0);
        }
        return Item{name(h), ix, hash};
    }
};

void decode_range(const uint8_t* buf, const uint64_t* offsets, uint32_t codec, bool strict, bool want_kv,
                  bool want_ann, DecodeRange* d) {
    std::vector<uint8_t> scratch;
    SpanT s;
    std::vector<const Ann*> distinct;
    d->recs.reserve(d->hi - d->lo);
    for (uint64_t i = d->lo; i < d->hi; ++i) {
        if (offsets[i + 1] < offsets[i]) {
            d->err_index = i;
            d->err_status = ZK_ERR_INVALID_ARG;
            d->err = "offsets not ascending at span " + std::to_string(i);
            return;
        }
        const uint8_t* p = buf + offsets[i];
        uint64_t len = offsets[i + 1] - offsets[i];
        if (codec == ZK_CODEC_SNAPPY_THRIFT) {
            if (!snappy_uncompress(p, len, &scratch)) {
                if (strict) {
                    d->err_index = i;
                    d->err_status = ZK_ERR_INVALID_SPAN;
                    d->err = "span " + std::to_string(i) + ": corrupt snappy block";
                    return;
                }
                ++d->rejected;
                continue;
            }
            p = scratch.data();
            len = scratch.size();
        }
        s.clear();
        Rd r{p, p + len};
        const char* why = nullptr;
        if (!read_span(r, &s))
            why = "undecodable thrift span";
        else if (!s.has_name)
            why = "No name set in Span";  // IncompleteTraceDataException (thrift.scala:101-104)
        else
            for (const Ann& a : s.anns) {
                if (a.ts <= 0) {
                    why = "Annotation must have a timestamp";  // thrift.scala:66-67
                    break;
                }
                if (a.value && a.value_len == 0) {
                    why = "Annotation must have a value";  // thrift.scala:69-70
                    break;
                }
            }
        if (why) {
            if (strict) {
                d->err_index = i;
                d->err_status = ZK_ERR_INVALID_SPAN;
                d->err = "span " + std::to_string(i) + ": " + why;
                return;
            }
            ++d->rejected;
            continue;
        }
        // ---- the record ----
        uint32_t f = s.has_parent ? ZK_F_HAS_PARENT : 0u;
        int64_t first = 0, last = 0;
        uint32_t cnt[4] = {0, 0, 0, 0};  // cs, cr, sr, ss
        const Host* srv = nullptr;
        const Host* cli = nullptr;
        for (size_t q = 0; q < s.anns.size(); ++q) {
            const Ann& a = s.anns[q];
            if (q == 0 || a.ts < first) first = a.ts;
            if (q == 0 || a.ts > last) last = a.ts;
            if (is_core(a.value, a.value_len)) {
                const int c = a.value[0] == 'c' ? (a.value[1] == 's' ? 0 : 1) : (a.value[1] == 'r' ? 2 : 3);
                if (cnt[c] < 2) ++cnt[c];
                if (a.host.present) {
                    if (c >= 2 && !srv) srv = &a.host;
                    if (c < 2 && !cli) cli = &a.host;
                }
            }
        }
        if (!s.anns.empty()) f |= ZK_F_HAS_ANNOTATIONS;
        int32_t svc = -1;
        if (srv) {
            f |= ZK_F_SVC_SERVER;
            svc = d->name(*srv);
        } else if (cli) {
            f |= ZK_F_SVC_CLIENT;
            svc = d->name(*cli);
        }
        f |= (cnt[0] << ZK_F_CS_SHIFT) | (cnt[1] << ZK_F_CR_SHIFT) | (cnt[2] << ZK_F_SR_SHIFT) | (cnt[3] << ZK_F_SS_SHIFT);
        Decoded rec{i, (uint64_t)s.trace_id, (uint64_t)s.id, s.has_parent ? (uint64_t)s.parent_id : 0ull,
                    s.anns.empty() ? 0 : first, s.anns.empty() ? 0 : last, f, svc,
                    (uint32_t)d->kv.size(), 0u, (uint32_t)d->ann.size(), 0u};
        // ---- indexer items: only spans with a last annotation (CassieSpanStore.scala:214-218) ----
        if (!s.anns.empty()) {
            if (want_kv)
                for (const BinAnn& b : s.banns)  // :235-241 one per binary annotation with a host
                    if (b.host.present) d->kv.push_back(d->item(b.host, b.key, b.key_len));
            if (want_ann) {
                // :222-233 non-core annotations grouped by value; the group's min (Annotation.compare:
                // (a.timestamp - b.timestamp).toInt, Annotation.scala:36-38; min keeps the first of
                // equals) yields one item if it has a host
                distinct.clear();
                for (const Ann& a : s.anns) {
                    if (is_core(a.value, a.value_len)) continue;
                    bool seen = false;
                    for (const Ann*& dd : distinct) {
                        if (dd->value_len == a.value_len &&
                            (a.value_len == 0 || memcmp(dd->value, a.value, a.value_len) == 0) &&
                            (dd->value == nullptr) == (a.value == nullptr)) {
                            if ((int32_t)(uint32_t)((uint64_t)dd->ts - (uint64_t)a.ts) > 0) dd = &a;  // truncated compare
                            seen = true;
                            break;
                        }
                    }
                    if (!seen) distinct.push_back(&a);
                }
                for (const Ann* a : distinct)
                    if (a->host.present) d->ann.push_back(d->item(a->host, a->value, a->value_len));
            }
        }
        rec.kv_n = (uint32_t)d->kv.size() - rec.kv0;
        rec.ann_n = (uint32_t)d->ann.size() - rec.ann0;
        d->recs.push_back(rec);
    }
}

// The decode threads of one zk_ingest, kept across calls (starting 15 threads per batch would cost
// about as much as decoding a small one) and joined when the decoder is destroyed. run(T, fn) calls
// fn(t) for every t < T -- t = 0 on the calling thread -- and returns when all are done; ranges
// without a worker (a thread that could not start) run on the calling thread.
class DecodePool {
  public:
    DecodePool() = default;
    DecodePool(const DecodePool&) = delete;
    DecodePool& operator=(const DecodePool&) = delete;
    ~DecodePool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    void run(uint32_t T, const std::function<void(uint32_t)>& fn) {
        if (T <= 1) {
            fn(0);
            return;
        }
        while (workers_.size() < T - 1) {
            const uint32_t idx = (uint32_t)workers_.size() + 1;
            try {
                workers_.emplace_back([this, idx] { loop(idx); });
            } catch (...) {
                break;
            }
        }
        const uint32_t nw = (uint32_t)workers_.size() < T - 1 ? (uint32_t)workers_.size() : T - 1;
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = &fn;
            width_ = nw;
            pending_ = nw;
            ++gen_;
        }
        cv_.notify_all();
        for (uint32_t t = nw + 1; t < T; ++t) fn(t);
        fn(0);
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [&] { return pending_ == 0; });
        job_ = nullptr;
    }

  private:
    void loop(uint32_t idx) {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(uint32_t)>* job;
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                if (idx > width_) continue;  // not part of this run
                job = job_;
            }
            (*job)(idx);
            std::lock_guard<std::mutex> lk(m_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(uint32_t)>* job_ = nullptr;
    uint32_t width_ = 0, pending_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

struct zk_ingest {
    std::unordered_map<std::string, uint32_t> svc_ids;
    std::vector<std::string> svc_names;
    std::unordered_map<uint64_t, std::string> strings;
    std::string err;
    DecodePool pool;

    uint32_t service(const Host& h) {
        // thrift.scala:36-43: null or "" service name -> Endpoint.UnknownServiceName
        std::string name = (h.svc && h.svc_len) ? std::string(h.svc, h.svc_len) : std::string(kUnknownService);
        auto it = svc_ids.find(name);
        if (it != svc_ids.end()) return it->second;
        const uint32_t id = (uint32_t)svc_names.size();
        svc_ids.emplace(name, id);
        svc_names.push_back(std::move(name));
        return id;
    }
    uint32_t exact(std::string name) {  // Service(name) as is (no "Unknown service name" rule)
        auto it = svc_ids.find(name);
        if (it != svc_ids.end()) return it->second;
        const uint32_t id = (uint32_t)svc_names.size();
        svc_ids.emplace(name, id);
        svc_names.push_back(std::move(name));
        return id;
    }
    void keep(uint64_t h, const std::string& s) {  // the string behind a hash (the first one seen)
        if (strings.find(h) == strings.end()) strings.emplace(h, s);
    }
};

extern "C" {

uint64_t zk_hash_string(const char* s, uint64_t len) {
    uint64_t h = 0xCBF29CE484222325ull;  // FNV-1a 64
    for (uint64_t i = 0; s && i < len; ++i) {
        h ^= (uint8_t)s[i];
        h *= 0x100000001B3ull;
    }
    return mix64(h);
}

zk_status zk_snappy_uncompress(const uint8_t* in, uint64_t in_len, uint8_t* out, uint64_t cap, uint64_t* out_len) {
    ZK_GUARD_BEGIN
    if (!in || !out_len) return ZK_ERR_INVALID_ARG;
    uint64_t len, hdr;
    if (!snappy_len(in, in_len, &len, &hdr) || !snappy_len_ok(len, in_len, hdr)) return ZK_ERR_INVALID_SPAN;
    *out_len = len;
    if (!out) return ZK_OK;
    if (cap < len) return ZK_ERR_CAPACITY;
    std::vector<uint8_t> tmp;
    if (!snappy_uncompress(in, in_len, &tmp)) return ZK_ERR_INVALID_SPAN;
    memcpy(out, tmp.data(), len);
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_ingest_create(zk_ingest** out) {
    ZK_GUARD_BEGIN
    if (!out) return ZK_ERR_INVALID_ARG;
    *out = new zk_ingest();
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_ingest_destroy(zk_ingest* g) {
    ZK_GUARD_BEGIN
    if (!g) return ZK_ERR_INVALID_ARG;
    delete g;
    return ZK_OK;
    ZK_GUARD_END
}

const char* zk_ingest_last_error(const zk_ingest* g) { return g ? g->err.c_str() : "null decoder"; }

zk_status zk_ingest_spans(zk_ingest* g, const uint8_t* buf, const uint64_t* offsets, uint64_t n, uint32_t codec,
                          uint32_t flags, const zk_span_cols* out, uint64_t* n_out, uint64_t* n_rejected,
                          zk_ingest_items* items) {
    ZK_GUARD_BEGIN
    if (!g || !n_out || !n_rejected) return ZK_ERR_INVALID_ARG;
    *n_out = *n_rejected = 0;
    if (items) items->kv_n = items->ann_n = 0;
    if (n == 0) return ZK_OK;
    if (!buf || !offsets || !out || !out->trace_id || !out->span_id || !out->parent_id || !out->first_ts ||
        !out->last_ts || !out->service_id || !out->flags)
        return ZK_ERR_INVALID_ARG;
    if (codec != ZK_CODEC_THRIFT && codec != ZK_CODEC_SNAPPY_THRIFT) {
        g->err = "unknown codec";
        return ZK_ERR_INVALID_ARG;
    }
    const bool strict = (flags & ZK_INGEST_STRICT) != 0;
    const bool want_kv = items && items->kv_service && items->kv_key;
    const bool want_ann = items && items->ann_service && items->ann_value;
    // Phase 1, in parallel over contiguous fragment ranges: decode and validate every fragment into
    // a thread-local list (names copied into the thread's own table). Phase 2, in input order on
    // this thread: assign service ids (in order of first appearance, exactly as a one-pass decode
    // would), write the records and items, intern the strings, stop at the first error.
    uint32_t T = std::thread::hardware_concurrency();
    T = T < 1 ? 1 : T > kIngestThreads ? kIngestThreads : T;
    if (flags & ZK_INGEST_ONE_THREAD) T = 1;
    if (n / kIngestMinPerThread < T) T = (uint32_t)(n / kIngestMinPerThread) > 1 ? (uint32_t)(n / kIngestMinPerThread) : 1;
    std::vector<DecodeRange> part(T);
    const std::function<void(uint32_t)> work = [&](uint32_t t) noexcept {  // (nothing may escape a worker thread)
        DecodeRange& d = part[t];
        d.lo = n * t / T;
        d.hi = n * (t + 1) / T;
        try {
            decode_range(buf, offsets, codec, strict, want_kv, want_ann, &d);
        } catch (...) {
            d.err_index = d.lo;
            d.err_status = ZK_ERR_CAPACITY;
            d.err = "host allocation failed";
        }
    };
    g->pool.run(T, work);
    uint64_t* o_tid = (uint64_t*)out->trace_id;
    uint64_t* o_sid = (uint64_t*)out->span_id;
    uint64_t* o_pid = (uint64_t*)out->parent_id;
    int64_t* o_first = (int64_t*)out->first_ts;
    int64_t* o_last = (int64_t*)out->last_ts;
    uint32_t* o_svc = (uint32_t*)out->service_id;
    uint32_t* o_flags = (uint32_t*)out->flags;
    bool item_overflow = false;
    uint64_t k = 0;
    for (uint32_t t = 0; t < T; ++t) {
        DecodeRange& d = part[t];
        std::vector<int64_t> gid(d.names.size(), -1);
        auto id_of = [&](int32_t name) -> uint32_t {
            if (gid[name] < 0) gid[name] = g->exact(d.names[name]);
            return (uint32_t)gid[name];
        };
        std::vector<uint8_t> kept(d.strs.size(), 0);  // strings of this range already interned
        auto keep = [&](const Item& it) {
            if (kept[it.str]) return;
            kept[it.str] = 1;
            g->keep(it.hash, d.strs[it.str]);
        };
        for (const Decoded& r : d.recs) {
            if (r.index >= d.err_index) break;  // records after this range's first error are not committed
            uint32_t svc = 0;
            if (r.svc_name >= 0) svc = id_of(r.svc_name);
            o_tid[k] = r.tid;
            o_sid[k] = r.sid;
            o_pid[k] = r.pid;
            o_first[k] = r.first;
            o_last[k] = r.last;
            o_svc[k] = svc;
            o_flags[k] = r.flags;
            ++k;
            for (uint32_t q = r.kv0; q < r.kv0 + r.kv_n; ++q) {  // :235-241 one per binary annotation with a host
                if (items->kv_n >= items->kv_cap) {
                    item_overflow = true;
                    continue;
                }
                const Item& it = d.kv[q];
                items->kv_service[items->kv_n] = id_of(it.name);
                items->kv_key[items->kv_n] = it.hash;
                keep(it);
                ++items->kv_n;
            }
            for (uint32_t q = r.ann0; q < r.ann0 + r.ann_n; ++q) {
                if (items->ann_n >= items->ann_cap) {
                    item_overflow = true;
                    continue;
                }
                const Item& it = d.ann[q];
                items->ann_service[items->ann_n] = id_of(it.name);
                items->ann_value[items->ann_n] = it.hash;
                keep(it);
                ++items->ann_n;
            }
        }
        *n_rejected += d.rejected;
        if (d.err_index != UINT64_MAX) {  // the first error of the batch (ranges are in input order)
            g->err = d.err;
            return d.err_status;
        }
    }
    *n_out = k;
    if (item_overflow) {
        g->err = "item buffer too small";
        return ZK_ERR_CAPACITY;
    }
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_ingest_num_services(const zk_ingest* g, uint32_t* n) {
    ZK_GUARD_BEGIN
    if (!g || !n) return ZK_ERR_INVALID_ARG;
    *n = (uint32_t)g->svc_names.size();
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_ingest_service_id(zk_ingest* g, const char* name, uint64_t len, uint32_t* id) {
    ZK_GUARD_BEGIN
    if (!g || !id || (!name && len)) return ZK_ERR_INVALID_ARG;
    Host h;
    h.present = true;
    h.svc = name;
    h.svc_len = (uint32_t)len;
    *id = g->service(h);
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_ingest_service_name(const zk_ingest* g, uint32_t id, char* buf, uint64_t cap, uint64_t* len) {
    ZK_GUARD_BEGIN
    if (!g || !len) return ZK_ERR_INVALID_ARG;
    if (id >= g->svc_names.size()) return ZK_ERR_SERVICE_RANGE;
    const std::string& s = g->svc_names[id];
    *len = s.size();
    if (!buf) return ZK_OK;
    if (cap < s.size()) return ZK_ERR_CAPACITY;
    memcpy(buf, s.data(), s.size());
    return ZK_OK;
    ZK_GUARD_END
}

// ---- Dependencies wire format (zipkinDependencies.thrift:24-43, ScroogeThriftCodec) -------------
zk_status zk_dependencies_encode(int64_t start_us, int64_t end_us, const zk_dep_link* links, uint64_t n_links,
                                 const char* const* names, const uint32_t* name_lens, uint32_t num_names,
                                 uint8_t* out, uint64_t cap, uint64_t* len) {
    ZK_GUARD_BEGIN
    if (!len || (n_links && !links) || (num_names && (!names || !name_lens))) return ZK_ERR_INVALID_ARG;
    if (n_links > 0x7FFFFFFFull) return ZK_ERR_INVALID_ARG;
    for (uint64_t i = 0; i < n_links; ++i)
        if (links[i].parent >= num_names || links[i].child >= num_names) return ZK_ERR_SERVICE_RANGE;
    Wr w{out, out ? cap : 0};
    // Dependencies {1: i64 start_time, 2: i64 end_time, 3: list<DependencyLink> links}
    w.i64(1, start_us);
    w.i64(2, end_us);
    w.field(T_LIST, 3);
    w.u8(T_STRUCT);
    w.be((uint32_t)n_links, 4);
    for (uint64_t i = 0; i < n_links; ++i) {
        const zk_dep_link& l = links[i];
        // DependencyLink {1: string parent, 2: string child, 3: Moments duration_moments}
        w.str(1, names[l.parent], name_lens[l.parent]);
        w.str(2, names[l.child], name_lens[l.child]);
        w.field(T_STRUCT, 3);
        // Moments {1: i64 m0, 2..5: double m1..m4}
        w.i64(1, l.moments.m0);
        w.dbl(2, l.moments.m1);
        w.dbl(3, l.moments.m2);
        w.dbl(4, l.moments.m3);
        w.dbl(5, l.moments.m4);
        w.u8(T_STOP);
        w.u8(T_STOP);
    }
    w.u8(T_STOP);
    *len = w.len;
    if (out && w.len > cap) return ZK_ERR_CAPACITY;
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_dependencies_decode(zk_ingest* g, const uint8_t* buf, uint64_t len, int64_t* start_us,
                                 int64_t* end_us, zk_dep_link* out, uint64_t cap, uint64_t* n_links) {
    ZK_GUARD_BEGIN
    if (!g || !buf || !start_us || !end_us || !n_links) return ZK_ERR_INVALID_ARG;
    Rd r{buf, buf + len};
    int64_t st = 0, en = 0;  // absent fields keep the thrift defaults
    uint64_t k = 0;
    bool overflow = false;
    for (;;) {
        const uint8_t t = r.u8();
        if (!r.ok || t == T_STOP) break;
        const int16_t id = r.i16();
        if (id == 1 && t == T_I64) {
            st = r.i64();
        } else if (id == 2 && t == T_I64) {
            en = r.i64();
        } else if (id == 3 && t == T_LIST) {
            const uint8_t et = r.u8();
            const int32_t n = r.i32();
            if (!r.ok || n < 0) break;
            if (et != T_STRUCT) {
                for (int32_t q = 0; r.ok && q < n; ++q) r.skip(et);
                continue;
            }
            for (int32_t q = 0; r.ok && q < n; ++q) {
                std::string parent, child;
                zk_moments m = {0, 0.0, 0.0, 0.0, 0.0};
                for (;;) {
                    const uint8_t lt = r.u8();
                    if (!r.ok || lt == T_STOP) break;
                    const int16_t lid = r.i16();
                    const char* s;
                    uint32_t sl;
                    if ((lid == 1 || lid == 2) && lt == T_STRING) {
                        if (r.str(&s, &sl)) (lid == 1 ? parent : child).assign(s, sl);
                    } else if (lid == 3 && lt == T_STRUCT) {
                        for (;;) {
                            const uint8_t mt = r.u8();
                            if (!r.ok || mt == T_STOP) break;
                            const int16_t mid = r.i16();
                            if (mid == 1 && mt == T_I64)
                                m.m0 = r.i64();
                            else if (mid >= 2 && mid <= 5 && mt == T_DOUBLE)
                                (mid == 2 ? m.m1 : mid == 3 ? m.m2 : mid == 4 ? m.m3 : m.m4) = bits_double(r.i64());
                            else
                                r.skip(mt);
                        }
                    } else {
                        r.skip(lt);
                    }
                }
                if (!r.ok) break;
                if (out && k < cap) {
                    out[k].parent = g->exact(parent);
                    out[k].child = g->exact(child);
                    out[k].moments = m;
                } else if (out) {
                    overflow = true;
                }
                ++k;
            }
        } else {
            r.skip(t);
        }
        if (!r.ok) break;
    }
    if (!r.ok) {
        g->err = "undecodable thrift Dependencies";
        return ZK_ERR_INVALID_SPAN;
    }
    *start_us = st;
    *end_us = en;
    *n_links = k;
    return overflow ? ZK_ERR_CAPACITY : ZK_OK;
    ZK_GUARD_END
}

int64_t zk_dependencies_row_key(int64_t start_us) {
    // Time.floor(1.day) (twitter util: integer division of the time, i.e. toward zero)
    constexpr int64_t kDayUs = 86400LL * 1000000LL;
    return (start_us / kDayUs) * kDayUs;
}

zk_status zk_ingest_string(const zk_ingest* g, uint64_t hash, char* buf, uint64_t cap, uint64_t* len) {
    ZK_GUARD_BEGIN
    if (!g || !len) return ZK_ERR_INVALID_ARG;
    auto it = g->strings.find(hash);
    if (it == g->strings.end()) return ZK_ERR_INVALID_ARG;
    *len = it->second.size();
    if (!buf) return ZK_OK;
    if (cap < it->second.size()) return ZK_ERR_CAPACITY;
    memcpy(buf, it->second.data(), it->second.size());
    return ZK_OK;
    ZK_GUARD_END
}

}  // extern "C"
