// zk_ingest_dev.hip — the span ingest decoder on the device (include/zkingest.h, zk_ingest_dev_*).
//
// The same contract as the host decoder (zk_ingest.cpp): stored fragments
// Snappy(TBinaryProtocol(thrift Span)) (CassieSpanStore.scala:52; SnappyCodec.scala:32-51;
// zipkinCore.thrift:27-58) -> thrift.scala validation (:36-121) -> the 48-B record of SURVEY
// Appendix A.1, written straight into HBM columns. One lane per fragment: the Snappy block and the
// thrift walk are sequential within a fragment, fragments are independent.
//
//   D2 k_ing_decode_lds per fragment: its extent and Snappy header (the uncompressed length, loaded
//                       one round ahead), decompress in LDS, walk the Span, validate, derive the
//                       record and the service name (FNV-1a 64 + splitmix64 of its bytes, as
//                       zk_hash_string); k_ing_decode takes the fragments it defers, in global
//                       memory, with scratch bump-allocated from one counter
//   D3 k_ing_dict_insert  claim a slot per new service hash in the persistent open-addressing table
//   (host)              give new slots ids in slot order and copy their names to the device arena
//   D4 k_ing_lookup     service hash -> id, the name bytes compared with the arena's (exact)
//   (hipcub scan)       of accepted records -> output positions
//   D5 k_ing_compact    accepted records -> the caller's columns, input order kept
//
// Every byte read is bounds-checked: corrupt input marks the fragment undecodable, never faults.
#include <string.h>

#include <algorithm>

#include <hipcub/hipcub.hpp>
#include <string>
#include <unordered_map>
#include <vector>

#include "zk_guard.h"
#include "zk_launch.h"
#include "zkingest.h"

namespace zk {
namespace {

constexpr uint32_t kIngWG = 256;
constexpr uint32_t kMaxRaw = ZK_INGEST_MAX_FRAGMENT;  // largest uncompressed fragment accepted (16 MiB)
constexpr uint64_t kEmpty = 0ull;            // empty dictionary slot (hash 0 is stored as 1)
constexpr uint32_t kNoId = 0xFFFFFFFFu;
// kStDefer: the global-memory kernel decodes it; kStNoScratch: the scratch ran out, decoded again
// after it grows (neither is left when the batch ends)
constexpr uint8_t kStOk = 0, kStInvalid = 1, kStUndecodable = 2, kStCollision = 3, kStRange = 4, kStDefer = 5,
                  kStNoScratch = 6;
const char kUnknown[] = "Unknown service name";  // Endpoint.UnknownServiceName (thrift.scala:36-43)

enum : uint8_t { T_STOP = 0, T_BOOL = 2, T_BYTE = 3, T_DOUBLE = 4, T_I16 = 6, T_I32 = 8, T_I64 = 10,
                 T_STRING = 11, T_STRUCT = 12, T_MAP = 13, T_SET = 14, T_LIST = 15 };

__device__ __forceinline__ uint64_t d_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t d_hash(const uint8_t* s, uint32_t n) {  // == zk_hash_string
    uint64_t h = 0xCBF29CE484222325ull;
    // 16 bytes' loads issued before the multiply chain consumes them (one round trip per 16 bytes
    // instead of one per byte)
    for (uint32_t i0 = 0; i0 < n; i0 += 16) {
        uint8_t v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = i0 + j < n ? s[i0 + j] : 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (i0 + j < n) {
                h ^= v[j];
                h *= 0x100000001B3ull;
            }
        }
    }
    h = d_mix64(h);
    return h ? h : 1ull;
}

typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;

// Multi-byte reads at any byte offset. Global / generic pointers: one unaligned access. LDS: an
// access off its natural alignment is replayed on gfx950 (cdna_hip_programming.md Guideline 17;
// SQ_LDS_UNALIGNED_STALL was 23 % of the LDS decoder's cycles, and splitting the 8-byte reads into
// unaligned 4-byte ones made it worse, profiles/r03/ingest_pmc.txt), so LDS bytes are read as
// ALIGNED dwords and shifted into place with v_alignbyte_b32.
template <class P>
__device__ __forceinline__ uint32_t ld_u32(P p) {
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}
__device__ __forceinline__ uint32_t ld_u32(const lds_u8* p) {
    const uint32_t a = (uint32_t)(uintptr_t)p;
    const lds_u32* w = (const lds_u32*)(uintptr_t)(a & ~3u);
    return __builtin_amdgcn_alignbyte(w[1], w[0], a & 3u);
}
template <class P>
__device__ __forceinline__ uint64_t ld_u64(P p) {
    uint64_t v;
    __builtin_memcpy(&v, p, 8);
    return v;
}
__device__ __forceinline__ uint64_t ld_u64(const lds_u8* p) {
    const uint32_t a = (uint32_t)(uintptr_t)p;
    const lds_u32* w = (const lds_u32*)(uintptr_t)(a & ~3u);
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], s = a & 3u;
    return ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, s) << 32) | __builtin_amdgcn_alignbyte(w1, w0, s);
}
__device__ __forceinline__ uint32_t ld_u32(lds_u8* p) { return ld_u32((const lds_u8*)p); }
__device__ __forceinline__ uint64_t ld_u64(lds_u8* p) { return ld_u64((const lds_u8*)p); }
template <class P>
__device__ __forceinline__ uint16_t ld_be16(P p) {
    return __builtin_bswap16((uint16_t)ld_u32(p));
}
template <class P>
__device__ __forceinline__ uint32_t ld_be32(P p) {
    return __builtin_bswap32(ld_u32(p));
}
template <class P>
__device__ __forceinline__ uint64_t ld_be64(P p) {
    return __builtin_bswap64(ld_u64(p));
}
// copy 8 / 4 bytes through a register (source read before the destination is written)
template <class D, class S>
__device__ __forceinline__ void cp8(D d, S s) {
    const uint64_t v = ld_u64(s);
    __builtin_memcpy(d, &v, 8);
}
template <class S>
__device__ __forceinline__ void cp8(lds_u8* d, S s) {
    // LDS destinations written byte by byte (never off alignment: unaligned stores replay),
    // 14.00 vs 14.03-14.21 ms per decode (profiles/r03/ingest_pmc.txt)
    const uint64_t v = ld_u64(s);
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = (uint8_t)(v >> (8 * k));
}
template <class D, class S>
__device__ __forceinline__ void cp4(D d, S s) {
    const uint32_t v = ld_u32(s);
    __builtin_memcpy(d, &v, 4);
}

// bounds-checked big-endian reader over [p, e); P is a generic pointer, or an LDS one (the LDS
// decoder: its reads are then ds_read_* instead of flat loads through the aperture)
template <class P>
struct DRdT {
    P p;
    P e;
    bool ok;
    __device__ bool need(uint64_t k) {
        if (!ok || (uint64_t)(e - p) < k) ok = false;
        return ok;
    }
    __device__ uint8_t u8() { return need(1) ? *p++ : 0; }
    __device__ int16_t i16() {
        if (!need(2)) return 0;
        const int16_t v = (int16_t)ld_be16(p);
        p += 2;
        return v;
    }
    __device__ int32_t i32() {
        if (!need(4)) return 0;
        const uint32_t v = ld_be32(p);
        p += 4;
        return (int32_t)v;
    }
    // a struct field header: its type, and its id unless the type is STOP (returns false then, or
    // on a short read). One 4-byte load when 4 bytes remain (the LDS decoder reads its fragment
    // with 32-bit loads instead of three byte loads per field).
    __device__ bool field(uint8_t* t, int16_t* id) {
        if (!ok) return false;
        if (e - p >= 4) {
            const uint32_t v = ld_be32(p);
            *t = (uint8_t)(v >> 24);
            if (*t == T_STOP) {
                p += 1;
                return false;
            }
            *id = (int16_t)(v >> 8);
            p += 3;
            return true;
        }
        *t = u8();
        if (!ok || *t == T_STOP) return false;
        *id = i16();
        return ok;
    }
    __device__ int64_t i64() {
        if (!need(8)) return 0;
        const uint64_t v = ld_be64(p);
        p += 8;
        return (int64_t)v;
    }
    __device__ bool str(P* s, uint32_t* len) {
        const int32_t l = i32();
        if (!ok || l < 0 || !need((uint64_t)l)) return ok = false;
        *s = p;
        *len = (uint32_t)l;
        p += l;
        return true;
    }
    // skip one value of type t; nested containers/structs iteratively up to a fixed depth
    __device__ void skip(uint8_t t) {
        // explicit stack: (type, remaining) for containers; structs use remaining = -1
        uint8_t st_t[16], st_k[16], st_v[16];
        int32_t st_n[16];
        int sp = 0;
        uint8_t cur = t;
        for (;;) {
            if (!ok) return;
            switch (cur) {
                case T_BOOL:
                case T_BYTE: u8(); break;
                case T_I16: i16(); break;
                case T_I32: i32(); break;
                case T_DOUBLE:
                case T_I64: i64(); break;
                case T_STRING: {
                    P s;
                    uint32_t l;
                    str(&s, &l);
                    break;
                }
                case T_STRUCT:
                case T_MAP:
                case T_SET:
                case T_LIST: {
                    if (sp == 16) {
                        ok = false;
                        return;
                    }
                    if (cur == T_STRUCT) {
                        st_t[sp] = T_STRUCT;
                        st_n[sp] = -1;
                    } else if (cur == T_MAP) {
                        st_t[sp] = T_MAP;
                        st_k[sp] = u8();
                        st_v[sp] = u8();
                        const int32_t mc = i32();
                        st_n[sp] = (mc < 0 || mc > (1 << 29)) ? -1 : mc * 2;  // keys and values alternate
                    } else {
                        st_t[sp] = cur;
                        st_k[sp] = u8();
                        st_n[sp] = i32();
                    }
                    if (!ok || (st_t[sp] != T_STRUCT && st_n[sp] < 0)) {
                        ok = false;
                        return;
                    }
                    ++sp;
                    break;
                }
                default: ok = false; return;
            }
            // the next value to skip: from the innermost open container, closing finished ones
            for (;;) {
                if (sp == 0) return;
                const int q = sp - 1;
                if (st_t[q] == T_STRUCT) {
                    const uint8_t ft = u8();
                    if (!ok) return;
                    if (ft == T_STOP) {
                        --sp;
                        continue;
                    }
                    i16();
                    cur = ft;
                    break;
                }
                if (st_n[q] == 0) {
                    --sp;
                    continue;
                }
                const int32_t left = st_n[q]--;
                cur = st_t[q] == T_MAP ? ((left & 1) ? st_v[q] : st_k[q]) : st_k[q];
                break;
            }
        }
    }
};

using DRd = DRdT<const uint8_t*>;

// The generic skip out of line (nested containers are rare in stored spans): keeps its stack and
// switch out of the decoders' register budget. DRd travels by value, so nothing goes to scratch.
template <class P>
__device__ __noinline__ DRdT<P> skip_call(DRdT<P> r, uint8_t t) {
    r.skip(t);
    return r;
}

// skip one value: fixed-width fields and strings inline, anything else through skip_call
template <class P>
__device__ __forceinline__ void skip_flat(DRdT<P>& r, uint8_t t) {
    uint32_t w = 0;
    switch (t) {
        case T_BOOL:
        case T_BYTE: w = 1; break;
        case T_I16: w = 2; break;
        case T_I32: w = 4; break;
        case T_DOUBLE:
        case T_I64: w = 8; break;
        case T_STRING: {
            const int32_t l = r.i32();
            if (!r.ok || l < 0 || !r.need((uint64_t)l)) {
                r.ok = false;
                return;
            }
            r.p += l;
            return;
        }
        default: r = skip_call(r, t); return;
    }
    if (r.need(w)) r.p += w;
}

// skip a struct whose fields are flat or flat structs (BinaryAnnotation with its Endpoint host)
template <class P>
__device__ __forceinline__ void skip_struct2(DRdT<P>& r) {
    for (;;) {
        uint8_t t;
        int16_t fid;
        if (!r.field(&t, &fid)) return;
        if (t != T_STRUCT) {
            skip_flat(r, t);
            continue;
        }
        uint8_t u;
        int16_t uid;
        while (r.field(&u, &uid)) skip_flat(r, u);
        if (!r.ok) return;
    }
}

// Snappy copy of l bytes from off back: an 8-byte (off >= 8) or 4-byte (off >= 4) step never reads
// what it writes; the overlapping rest goes bytewise
template <class P>
__device__ __forceinline__ void backref_copy(P out, uint64_t o, uint64_t off, uint64_t l) {
    uint64_t k = 0;
    if (off >= 8) {
        for (; k + 8 <= l; k += 8) cp8(out + o + k, out + o - off + k);
    } else if (off >= 4) {
        for (; k + 4 <= l; k += 4) cp4(out + o + k, out + o - off + k);
    }
    #pragma clang loop vectorize(disable)  // (a vectorised byte loop reads LDS with unaligned ds_read_b128)
    for (; k < l; ++k) out[o + k] = out[o - off + k];
}

template <class P>
__device__ __forceinline__ bool snappy_hdr(P in, uint64_t n, uint64_t* len, uint64_t* hdr) {
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

__device__ __forceinline__ bool snappy_block(const uint8_t* in, uint64_t n, uint8_t* out, uint64_t len) {
    uint64_t dl, hdr;
    if (!snappy_hdr(in, n, &dl, &hdr) || dl != len) return false;
    uint64_t o = 0, i = hdr;
    while (i < n) {
        const uint8_t tag = in[i++];
        uint64_t l, off;
        const uint32_t kind = tag & 3;
        if (kind == 0) {
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
            uint64_t k = 0;
            for (; k + 8 <= l; k += 8) cp8(out + o + k, in + i + k);
            #pragma clang loop vectorize(disable)  // (a vectorised byte loop reads LDS with unaligned ds_read_b128)
            for (; k < l; ++k) out[o + k] = in[i + k];
            i += l;
            o += l;
            continue;
        }
        if (kind == 1) {
            if (i + 1 > n) return false;
            l = ((tag >> 2) & 7) + 4;
            off = ((uint64_t)(tag >> 5) << 8) | in[i];
            i += 1;
        } else if (kind == 2) {
            if (i + 2 > n) return false;
            l = (tag >> 2) + 1;
            off = (uint64_t)in[i] | ((uint64_t)in[i + 1] << 8);
            i += 2;
        } else {
            if (i + 4 > n) return false;
            l = (tag >> 2) + 1;
            off = (uint64_t)in[i] | ((uint64_t)in[i + 1] << 8) | ((uint64_t)in[i + 2] << 16) |
                  ((uint64_t)in[i + 3] << 24);
            i += 4;
        }
        if (off == 0 || off > o || o + l > len) return false;
        backref_copy(out, o, off, l);
        o += l;
    }
    return o == len;
}

struct IngArgs {
    const uint8_t* buf;
    const uint64_t* offsets;  // fragment i: buf[offsets[i], ends[i])
    const uint64_t* ends;     // offsets + 1 for one batch; a separate array for several (ingest_multi)
    uint64_t n;
    uint32_t snappy;
    uint8_t* scratch;                   // Snappy: deferred fragments' Spans and copied-out names
    uint64_t scratch_cap;
    unsigned long long* scratch_used;   // bump counter (may run past scratch_cap: see kStNoScratch)
    // per-fragment results
    uint8_t* status;
    uint64_t* tid;
    uint64_t* sid;
    uint64_t* pid;
    int64_t* first;
    int64_t* last;
    uint32_t* flags;
    uint32_t* svc;       // dictionary id after D4
    uint64_t* svc_hash;  // 0: no service
    uint64_t* name_ptr;  // device address of the service name bytes
    uint32_t* name_len;
    uint32_t* keep;      // 1 = record goes to the output (n + 1 for the scan)
    uint32_t* pub;       // fragments that published a name for D3/D4 (count in *pub_n)
    unsigned long long* pub_n;
    uint32_t* def;       // fragments the LDS decoder deferred (count in *def_n)
    unsigned long long* def_n;
    unsigned long long* claims;  // dictionary slots D3 claimed in this batch
    uint32_t lds_block;          // fragments per wave of the LDS decoder
    uint32_t* pos;       // n + 1
    // dictionary
    uint64_t* d_key;
    uint32_t* d_id;
    uint64_t* d_ptr;     // device address of the slot's name (arena after assignment)
    uint32_t* d_len;
    const uint8_t* d_name16;  // the first 16 bytes of each named slot's name (zero padded), 16-B aligned
    uint32_t d_mask;
    uint32_t max_services;
    const uint8_t* unknown;  // device copy of kUnknown
    // ---- the span indexer's items (zk_ingest_dev_spans_items; items == 0: none) ----
    uint32_t items;
    uint32_t* kv_svc;            // item service: an id, or a reference resolved by k_ing_item_fixup
    uint64_t* kv_key;
    uint64_t kv_cap;
    uint32_t* an_svc;
    uint64_t* an_val;
    uint64_t an_cap;
    uint32_t* skip_kv;           // per fragment: items a failed attempt already appended
    uint32_t* skip_an;
    uint64_t* s_key;             // set of the key / value hashes whose strings are captured
    uint32_t s_mask;
    uint64_t* ns_hash;           // strings captured in this batch (hash, global bytes, length)
    uint64_t* ns_ptr;
    uint32_t* ns_len;
    uint64_t ns_cap;
    uint64_t* x_hash;            // item hosts not yet in the dictionary (published like a fragment's
    uint64_t* x_ptr;             // service name; D3 / D4 run over them as over fragments)
    uint32_t* x_len;
    uint32_t* x_svc;
    uint32_t* x_keep;
    uint8_t* x_status;
    uint32_t* x_list;
    uint64_t x_cap;
    unsigned long long* icnt;    // [0] / [1] kv / annotation items appended directly (the global-memory
                                 // decoder) [2] captured strings [3] extra names [4] attempts failed on a
                                 // full string set [5] / [6] extra-name collisions / range errors
                                 // [7] / [8] chunked items dropped (staging full) [9] / [10] chunked items
                                 // kept [11] / [12] chunks taken
    // the LDS decoder's items go to per-wave chunks of kItemChunk slots (one global atomic per chunk,
    // not per wave-append: every wave appending to one counter serialised on its L2 atomic unit),
    // compacted into the caller's buffers after the batch (k_ing_item_compact)
    uint32_t* ck_svc[2];
    uint64_t* ck_key[2];
    uint32_t* ck_fill[2];        // items in each chunk
    uint32_t ck_cap;             // chunks per kind
};

// A fragment's first bytes (its Snappy header varint is at most 5), issued as independent loads:
// one round trip. Bytes past the fragment read as 0x80 (a continuation), so they never end it.
__device__ __forceinline__ void head_bytes(const IngArgs& a, bool have, uint64_t b, uint64_t e, uint32_t h[5]) {
    const uint64_t n = have && a.snappy && e > b ? e - b : 0;
#pragma unroll
    for (int j = 0; j < 5; ++j) h[j] = (uint64_t)j < n ? a.buf[b + j] : 0x80u;
}

// D1 per fragment, as the host decoder's checks: offsets ascending; for Snappy a well-formed header
// whose length is at most kMaxRaw and at most ZK_SNAPPY_MAX_EXPANSION x the compressed bytes after it.
// *raw: the uncompressed length (0 for the thrift codec).
__device__ __forceinline__ uint8_t head_status(bool snappy, uint64_t b, uint64_t e, const uint32_t h[5], uint64_t* raw) {
    *raw = 0;
    if (e < b) return kStUndecodable;
    if (!snappy) return kStOk;
    uint64_t v = 0;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        v |= (uint64_t)(h[j] & 0x7Fu) << (7 * j);
        if (!(h[j] & 0x80u)) {
            if (v > kMaxRaw || v > (e - b - (uint64_t)(j + 1)) * (uint64_t)ZK_SNAPPY_MAX_EXPANSION) return kStUndecodable;
            *raw = v;
            return kStOk;
        }
    }
    return kStUndecodable;
}

// bytes of the scratch, or null when it is exhausted (the fragment is then marked kStNoScratch)
__device__ __forceinline__ uint8_t* scratch_take(const IngArgs& a, uint64_t bytes) {
    const unsigned long long off = atomicAdd(a.scratch_used, (unsigned long long)bytes);
    return off + bytes <= a.scratch_cap ? a.scratch + off : nullptr;
}

template <class P>
__device__ __forceinline__ bool is_core(P v, uint32_t l, int* c) {
    if (!v || l != 2) return false;
    if (v[0] == 'c' && (v[1] == 's' || v[1] == 'r')) {
        *c = v[1] == 's' ? 0 : 1;
        return true;
    }
    if (v[0] == 's' && (v[1] == 'r' || v[1] == 's')) {
        *c = v[1] == 'r' ? 2 : 3;
        return true;
    }
    return false;
}

// the service name of an endpoint struct: field 3 (string); absent or "" -> kUnknown. Like the
// host's read_endpoint, a second host field of the same annotation keeps the first one's name
// unless it has its own (the caller resets the name per annotation).
template <class P>
__device__ __forceinline__ void read_endpoint(DRdT<P>& r, P* name, uint32_t* nlen) {
    for (;;) {
        uint8_t t;
        int16_t id;
        if (!r.field(&t, &id)) return;
        if (id == 3 && t == T_STRING)
            r.str(name, nlen);
        else
            skip_flat(r, t);
    }
}

// The thrift walk of one decompressed Span at [src, src + len): validation (status on failure,
// -1), the record columns, and the service name (1: *nm/*nl set; 0: the span has no service).
template <class P>
__device__ __forceinline__ int parse_record(const IngArgs& a, uint64_t i, P src, uint64_t len,
                                            const uint8_t** nm_out, uint32_t* nl_out) {
    DRdT<P> r{src, src + len, true};
    int64_t trace = 0, id = 0, parent = 0;
    bool has_parent = false, has_name = false, invalid = false;
    int64_t first = 0, last = 0;
    uint32_t nann = 0, cnt[4] = {0, 0, 0, 0};
    P srv = nullptr;  // first sr/ss host's name (srv_set: a host was seen)
    P cli = nullptr;
    uint32_t srv_len = 0, cli_len = 0;
    bool srv_set = false, cli_set = false;
    for (;;) {
        uint8_t t;
        int16_t fid;
        if (!r.field(&t, &fid)) break;
        if (fid == 1 && t == T_I64) {
            trace = r.i64();
        } else if (fid == 3 && t == T_STRING) {
            P s;
            uint32_t l;
            has_name = r.str(&s, &l);
        } else if (fid == 4 && t == T_I64) {
            id = r.i64();
        } else if (fid == 5 && t == T_I64) {
            parent = r.i64();
            has_parent = true;
        } else if (fid == 6 && t == T_LIST) {
            const uint8_t et = r.u8();
            const int32_t cntl = r.i32();
            if (!r.ok || cntl < 0) {
                r.ok = false;
                break;
            }
            if (et != T_STRUCT) {
                for (int32_t q = 0; r.ok && q < cntl; ++q) skip_flat(r, et);
                continue;
            }
            for (int32_t q = 0; r.ok && q < cntl; ++q) {
                // Annotation {1: i64 timestamp, 2: string value, 3: optional Endpoint host}
                int64_t ts = 0;
                P v = nullptr;
                uint32_t vl = 0;
                bool host = false;
                P hn = nullptr;
                uint32_t hl = 0;
                for (;;) {
                    uint8_t at;
                    int16_t aid;
                    if (!r.field(&at, &aid)) break;
                    if (aid == 1 && at == T_I64)
                        ts = r.i64();
                    else if (aid == 2 && at == T_STRING)
                        r.str(&v, &vl);
                    else if (aid == 3 && at == T_STRUCT) {
                        host = true;
                        read_endpoint(r, &hn, &hl);
                    } else
                        skip_flat(r, at);
                }
                if (!r.ok) break;
                if (ts <= 0 || (v && vl == 0)) invalid = true;  // thrift.scala:66-71
                if (nann == 0 || ts < first) first = ts;
                if (nann == 0 || ts > last) last = ts;
                ++nann;
                int c;
                if (is_core(v, vl, &c)) {
                    if (cnt[c] < 2) ++cnt[c];
                    if (host) {
                        if (c >= 2 && !srv_set) {
                            srv_set = true;
                            srv = hn;
                            srv_len = hl;
                        }
                        if (c < 2 && !cli_set) {
                            cli_set = true;
                            cli = hn;
                            cli_len = hl;
                        }
                    }
                }
            }
        } else if (t == T_LIST) {  // binary_annotations (fid 8) and any other list
            const uint8_t et = r.u8();
            const int32_t cntl = r.i32();
            if (!r.ok || cntl < 0) {
                r.ok = false;
                break;
            }
            if (et == T_STRUCT)
                for (int32_t q = 0; r.ok && q < cntl; ++q) skip_struct2(r);
            else
                for (int32_t q = 0; r.ok && q < cntl; ++q) skip_flat(r, et);
        } else {
            skip_flat(r, t);
        }
        if (!r.ok) break;
    }
    if (!r.ok) {
        a.status[i] = kStUndecodable;
        return -1;
    }
    if (!has_name || invalid) {  // IncompleteTraceDataException / IllegalArgumentException
        a.status[i] = kStInvalid;
        return -1;
    }
    uint32_t f = has_parent ? ZK_F_HAS_PARENT : 0u;
    if (nann) f |= ZK_F_HAS_ANNOTATIONS;
    const uint8_t* nm = nullptr;
    uint32_t nl = 0;
    if (srv_set) {
        f |= ZK_F_SVC_SERVER;
        nm = (const uint8_t*)srv;
        nl = srv_len;
    } else if (cli_set) {
        f |= ZK_F_SVC_CLIENT;
        nm = (const uint8_t*)cli;
        nl = cli_len;
    }
    if ((srv_set || cli_set) && (!nm || nl == 0)) {
        nm = a.unknown;
        nl = sizeof(kUnknown) - 1;
    }
    f |= (cnt[0] << ZK_F_CS_SHIFT) | (cnt[1] << ZK_F_CR_SHIFT) | (cnt[2] << ZK_F_SR_SHIFT) | (cnt[3] << ZK_F_SS_SHIFT);
    a.tid[i] = (uint64_t)trace;
    a.sid[i] = (uint64_t)id;
    a.pid[i] = has_parent ? (uint64_t)parent : 0ull;
    a.first[i] = nann ? first : 0;
    a.last[i] = nann ? last : 0;
    a.flags[i] = f;
    a.svc[i] = 0u;
    *nm_out = nm;
    *nl_out = nl;
    return (srv_set || cli_set) ? 1 : 0;
}

// ---- the flat thrift walk (LDS decoder) -------------------------------------------------------
// parse_record's nested loops and switches compile to exec-mask bookkeeping (~250 saveexec/branch
// pairs and 210 SGPR spills in k_ing_decode_lds), and every lane pays for every path. The flat walk
// consumes ONE token per iteration -- a struct field header and its value, a list/set/map element,
// or a container end -- with the same straight-line code for every lane: one 16-byte LDS window at
// the cursor, the value's width and the semantic capture as selects, and a container push/pop on
// a 4-level register stack (span -> annotation list -> annotation -> endpoint; a span nested any
// deeper goes to the global-memory decoder, like an oversized one). Accept/reject and every captured value follow
// the host decoder (zk_ingest.cpp read_span / read_annotation / read_endpoint): last field wins,
// an annotation's host name is reset per annotation only.
// (A table-driven "flat" walk -- one token per step, every decision a select -- measured
// 15.6-15.9 ms per 1.98e7 fragments against 14.1-14.3 ms for this branchy walk, whose lanes hardly
// diverge on uniform layouts: profiles/r03/ingest_flat_walk.txt; removed after round 3.)

// ---- fast path: the canonical layout of a stored zipkin Span (LDS decoder) ----------------------
// Scrooge writes a Span's fields in id order (zipkinCore.thrift:27-58): 1 trace_id, 3 name, 4 id,
// 5 parent_id (optional), 6 annotations {1 timestamp, 2 value, 3 host (optional) {1 ipv4, 2 port,
// 3 service_name}}, 8 binary_annotations (optional) {1 key, 2 value, 3 annotation_type, 4 host
// (optional)}, 9 debug (optional). The branchy walk reads that as ~47 dependent tokens (a header
// byte, then the value, then the next header); here each group of fixed-layout fields is ONE
// window of aligned LDS dwords, checked byte for byte, so a span costs ~13 dependent steps (2 per
// annotation). Anything else -- another field, another order, a missing endpoint field, a length
// past the end -- returns -3 before anything is written, and the lane runs the generic walk: the
// fast path accepts only byte strings on which parse_record yields exactly the same record.
template <int W>
struct LWin {  // W + 1 aligned dwords from the dword holding byte x; byte x + j is at compile-time j
    uint32_t d[W + 1];
    uint32_t s;
    __device__ __forceinline__ void load(const lds_u8* base, uint32_t x) {
        const uint32_t adr = (uint32_t)(uintptr_t)(base + x);
        const lds_u32* w = (const lds_u32*)(uintptr_t)(adr & ~3u);
        s = adr & 3u;
#pragma unroll
        for (int k = 0; k <= W; ++k) d[k] = w[k];
    }
    template <int K>
    __device__ __forceinline__ uint32_t dw() const {  // bytes x + 4K .. x + 4K + 3
        static_assert(K + 1 <= W, "window too short");
        return __builtin_amdgcn_alignbyte(d[K + 1], d[K], s);
    }
    template <int J>
    __device__ __forceinline__ uint32_t raw32() const {  // bytes x + J .. x + J + 3, little-endian
        if constexpr ((J & 3) == 0)
            return dw<(J >> 2)>();
        else
            return (dw<(J >> 2)>() >> (8 * (J & 3))) | (dw<(J >> 2) + 1>() << (32 - 8 * (J & 3)));
    }
    template <int J>
    __device__ __forceinline__ uint32_t u8() const { return raw32<J>() & 0xFFu; }
    template <int J>
    __device__ __forceinline__ uint32_t be32() const { return __builtin_bswap32(raw32<J>()); }
    template <int J>
    __device__ __forceinline__ uint64_t be64() const { return ((uint64_t)be32<J>() << 32) | be32<J + 4>(); }
    template <int J>
    __device__ __forceinline__ uint32_t hdr() const { return be32<J>() >> 8; }  // type << 16 | field id
};
constexpr uint32_t fh(uint32_t type, uint32_t id) { return (type << 16) | id; }

// a length-prefixed value of `len` bytes after `at` header bytes fits the remaining `avail`
__device__ __forceinline__ bool fits(uint32_t avail, uint32_t at, int32_t len) {
    return len >= 0 && (uint64_t)avail >= (uint64_t)at + (uint32_t)len;
}

// lay (for the item walk): [0] the first annotation's offset, [1] their count, [2] the first binary
// annotation's offset, [3] their count
__device__ __forceinline__ int parse_record_fast(const IngArgs& a, uint64_t i, const lds_u8* base, uint32_t p0,
                                                 uint32_t len, uint32_t* nm_off, uint32_t* nl_out, uint32_t lay[4]) {
    constexpr int kNo = -3;
    const uint32_t e = p0 + len;
    uint32_t p = p0;
    // [0A 0001] trace_id [0B 0003] name
    LWin<5> w1;
    w1.load(base, p);
    if (e - p < 18u || w1.hdr<0>() != fh(T_I64, 1) || w1.hdr<11>() != fh(T_STRING, 3)) return kNo;
    const uint64_t trace = w1.be64<3>();
    const int32_t nlen = (int32_t)w1.be32<14>();
    if (!fits(e - p, 18u, nlen)) return kNo;
    p += 18u + (uint32_t)nlen;
    // [0A 0004] id, [0A 0005] parent_id (optional), [0F 0006] [0C] count
    LWin<8> w2;
    w2.load(base, p);
    if (e - p < 11u || w2.hdr<0>() != fh(T_I64, 4)) return kNo;
    const uint64_t id = w2.be64<3>();
    const bool has_parent = w2.hdr<11>() == fh(T_I64, 5);
    const uint64_t parent = w2.be64<14>();
    const uint32_t lh = has_parent ? w2.hdr<22>() : w2.hdr<11>();
    const uint32_t let = has_parent ? w2.u8<25>() : w2.u8<14>();
    const int32_t na = (int32_t)(has_parent ? w2.be32<26>() : w2.be32<15>());
    const uint32_t q2 = has_parent ? 30u : 19u;
    if (e - p < q2 || lh != fh(T_LIST, 6) || let != T_STRUCT || na < 0) return kNo;
    p += q2;
    lay[0] = p;
    lay[1] = (uint32_t)na;
    int64_t first = 0, last = 0;
    uint32_t nann = 0, cnt = 0;
    bool invalid = false, srv_set = false, cli_set = false;
    uint32_t srv = 0, srv_len = 0, cli = 0, cli_len = 0;
    for (int32_t k = 0; k < na; ++k) {
        // [0A 0001] timestamp [0B 0002] value
        LWin<6> c;
        c.load(base, p);
        if (e - p < 18u || c.hdr<0>() != fh(T_I64, 1) || c.hdr<11>() != fh(T_STRING, 2)) return kNo;
        const int64_t ts = (int64_t)c.be64<3>();
        const int32_t vl = (int32_t)c.be32<14>();
        if (!fits(e - p, 18u, vl)) return kNo;
        const uint32_t vc = c.raw32<18>() & 0xFFFFu;  // the value's first two bytes (used when vl == 2)
        p += 18u + (uint32_t)vl;
        // STOP, or [0C 0003] {[08 0001] ipv4 [06 0002] port [0B 0003] service_name} STOP STOP
        LWin<6> h;
        h.load(base, p);
        if (e - p < 1u) return kNo;
        bool host = false;
        uint32_t hn = 0, hl = 0;
        if (h.u8<0>() == T_STOP) {
            p += 1u;
        } else {
            if (e - p < 22u || h.hdr<0>() != fh(T_STRUCT, 3) || h.hdr<3>() != fh(T_I32, 1) ||
                h.hdr<10>() != fh(T_I16, 2) || h.hdr<15>() != fh(T_STRING, 3))
                return kNo;
            const int32_t L = (int32_t)h.be32<18>();
            if (!fits(e - p, 24u, L)) return kNo;  // + the two STOPs
            hn = p + 22u;
            hl = (uint32_t)L;
            host = true;
            p += 22u + (uint32_t)L;
            LWin<1> z;
            z.load(base, p);
            if ((z.raw32<0>() & 0xFFFFu) != 0u) return kNo;
            p += 2u;
        }
        // read_annotation returned: thrift.scala:66-71, Span.scala:213-240 (as parse_record)
        if (ts <= 0 || vl == 0) invalid = true;
        if (nann == 0u || ts < first) first = ts;
        if (nann == 0u || ts > last) last = ts;
        ++nann;
        const uint32_t c0 = vc & 0xFFu, c1 = vc >> 8;
        if (vl == 2 && ((c0 == 'c' && (c1 == 's' || c1 == 'r')) || (c0 == 's' && (c1 == 'r' || c1 == 's')))) {
            const uint32_t cc = c0 == 'c' ? (c1 == 's' ? 0u : 1u) : (c1 == 'r' ? 2u : 3u);
            if (((cnt >> (2 * cc)) & 3u) < 2u) cnt += 1u << (2 * cc);
            if (host && cc >= 2u && !srv_set) {
                srv_set = true;
                srv = hn;
                srv_len = hl;
            }
            if (host && cc < 2u && !cli_set) {
                cli_set = true;
                cli = hn;
                cli_len = hl;
            }
        }
    }
    // [0F 0008] [0C] count (optional)
    LWin<3> d;
    d.load(base, p);
    int32_t nb = 0;
    if (e - p >= 8u && d.hdr<0>() == fh(T_LIST, 8)) {
        nb = (int32_t)d.be32<4>();
        if (d.u8<3>() != T_STRUCT || nb < 0) return kNo;
        p += 8u;
    }
    lay[2] = p;
    lay[3] = (uint32_t)nb;
    for (int32_t k = 0; k < nb; ++k) {
        // [0B 0001] key [0B 0002] value [08 0003] annotation_type, then STOP or [0C 0004] endpoint STOP STOP
        LWin<2> k1;
        k1.load(base, p);
        if (e - p < 7u || k1.hdr<0>() != fh(T_STRING, 1)) return kNo;
        const int32_t kl = (int32_t)k1.be32<3>();
        if (!fits(e - p, 7u, kl)) return kNo;
        p += 7u + (uint32_t)kl;
        LWin<2> k2;
        k2.load(base, p);
        if (e - p < 7u || k2.hdr<0>() != fh(T_STRING, 2)) return kNo;
        const int32_t bl = (int32_t)k2.be32<3>();
        if (!fits(e - p, 7u, bl)) return kNo;
        p += 7u + (uint32_t)bl;
        LWin<8> k3;
        k3.load(base, p);
        if (e - p < 8u || k3.hdr<0>() != fh(T_I32, 3)) return kNo;
        if (k3.u8<7>() == T_STOP) {
            p += 8u;
        } else {
            if (e - p < 29u || k3.hdr<7>() != fh(T_STRUCT, 4) || k3.hdr<10>() != fh(T_I32, 1) ||
                k3.hdr<17>() != fh(T_I16, 2) || k3.hdr<22>() != fh(T_STRING, 3))
                return kNo;
            const int32_t L = (int32_t)k3.be32<25>();
            if (!fits(e - p, 31u, L)) return kNo;
            p += 29u + (uint32_t)L;
            LWin<1> z;
            z.load(base, p);
            if ((z.raw32<0>() & 0xFFFFu) != 0u) return kNo;
            p += 2u;
        }
    }
    // [02 0009] debug (optional), then the Span's STOP
    LWin<2> f;
    f.load(base, p);
    if (e - p < 1u) return kNo;
    if (f.u8<0>() != T_STOP) {
        if (e - p < 5u || f.hdr<0>() != fh(T_BOOL, 9) || f.u8<4>() != T_STOP) return kNo;
    }
    // the record (as parse_record: the name is present, so only the annotations can invalidate)
    if (invalid) {
        a.status[i] = kStInvalid;
        return -1;
    }
    uint32_t fl = has_parent ? ZK_F_HAS_PARENT : 0u;
    if (nann) fl |= ZK_F_HAS_ANNOTATIONS;
    *nm_off = ~0u;
    *nl_out = 0u;
    if (srv_set) {
        fl |= ZK_F_SVC_SERVER;
        if (srv_len) {
            *nm_off = srv;
            *nl_out = srv_len;
        }
    } else if (cli_set) {
        fl |= ZK_F_SVC_CLIENT;
        if (cli_len) {
            *nm_off = cli;
            *nl_out = cli_len;
        }
    }
    fl |= ((cnt & 3u) << ZK_F_CS_SHIFT) | (((cnt >> 2) & 3u) << ZK_F_CR_SHIFT) | (((cnt >> 4) & 3u) << ZK_F_SR_SHIFT) |
          (((cnt >> 6) & 3u) << ZK_F_SS_SHIFT);
    a.tid[i] = trace;
    a.sid[i] = id;
    a.pid[i] = has_parent ? parent : 0ull;
    a.first[i] = nann ? first : 0;
    a.last[i] = nann ? last : 0;
    a.flags[i] = fl;
    a.svc[i] = 0u;
    return (srv_set || cli_set) ? 1 : 0;
}

// ZK_ING_LISTS: the LDS decoder lists the fragments it defers and every decoder lists the
// fragments that publish a name, so the deferred decode, D3 and D4 visit those alone (after the
// first batches of a decoder both lists are empty) instead of sweeping all n fragments.
#ifndef ZK_ING_LISTS
#define ZK_ING_LISTS 1
#endif
// one atomic per wave: the active lanes take consecutive entries
__device__ __forceinline__ void list_add(uint32_t* list, unsigned long long* cnt, uint64_t i) {
    const unsigned long long mask = __ballot(1);
    const uint32_t lane = __lane_id();
    const uint32_t leader = (uint32_t)__ffsll(mask) - 1u;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(cnt, (unsigned long long)__popcll(mask));
    base = __shfl(base, (int)leader);
    list[base + (uint64_t)__popcll(mask & ((1ull << lane) - 1ull))] = (uint32_t)i;
}

__device__ __forceinline__ void publish_name(const IngArgs& a, uint64_t i, const uint8_t* nm, uint32_t nl) {
    a.svc_hash[i] = d_hash(nm, nl);
    a.name_ptr[i] = (uint64_t)(uintptr_t)nm;
    a.name_len[i] = nl;
#if ZK_ING_LISTS
    list_add(a.pub, a.pub_n, i);
#endif
}

// the fragment index of work item t of a list kernel (grid-stride over the list, or over all n)
#if ZK_ING_LISTS
#define ING_FOR_LIST(list, cnt, i)                                                              \
    const uint64_t ing_m = *(cnt);                                                              \
    for (uint64_t ing_t = (uint64_t)blockIdx.x * kIngWG + threadIdx.x; ing_t < ing_m;           \
         ing_t += (uint64_t)gridDim.x * kIngWG)                                                 \
        if (const uint64_t i = (list)[ing_t]; true)
#else
#define ING_FOR_LIST(list, cnt, i)                                                              \
    for (uint64_t i = (uint64_t)blockIdx.x * kIngWG + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * kIngWG)
#endif

// A name the dictionary already holds (an id assigned by an earlier batch) resolves right here:
// the slot of its hash, its bytes compared exactly with the arena's. svc_hash stays 0, so D3/D4
// skip the fragment. Anything else (a new name, a hash collision, an id out of range) is published
// for D3/D4, which decide it as before.
__device__ __forceinline__ bool try_resolve(const IngArgs& a, uint64_t i, const uint8_t* nm, uint32_t nl, uint64_t h) {
    uint32_t slot = (uint32_t)h & a.d_mask;
    for (uint32_t step = 0; step <= a.d_mask; ++step) {
        const uint64_t k = a.d_key[slot];
        if (k == kEmpty) return false;
        if (k == h) break;
        slot = (slot + 1) & a.d_mask;
    }
    if (a.d_key[slot] != h) return false;
    const uint32_t id = a.d_id[slot];
    if (id == kNoId || id >= a.max_services || a.d_len[slot] != nl) return false;
    const uint8_t* y = (const uint8_t*)(uintptr_t)a.d_ptr[slot];
    for (uint32_t q0 = 0; q0 < nl; q0 += 16) {  // 16 bytes of each side in flight at once
        uint8_t u[16], v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            u[j] = q0 + j < nl ? nm[q0 + j] : 0;
            v[j] = q0 + j < nl ? y[q0 + j] : 0;
        }
        bool eq = true;
#pragma unroll
        for (int j = 0; j < 16; ++j) eq &= u[j] == v[j];
        if (!eq) return false;
    }
    a.svc[i] = id;
    return true;
}

#ifndef ZK_ING_NAME16
#define ZK_ING_NAME16 1
#endif
// try_resolve for the LDS decoder in one global round trip for names of at most 16 bytes: the
// name's first 16 bytes are loaded once (hashed and compared from registers), and the first probe
// reads the slot's key, id, length and inline name bytes together. *h: the name's hash (for
// publish_name when it does not resolve).
__device__ __forceinline__ bool resolve16_id(const IngArgs& a, const uint8_t* nm, uint32_t nl, uint64_t* h_out,
                                             uint32_t* id_out) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    uint8_t u[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) u[j] = (uint32_t)j < nl ? nm[j] : 0;
    uint64_t h = 0xCBF29CE484222325ull;  // == d_hash
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        if ((uint32_t)j < nl) {
            h ^= u[j];
            h *= 0x100000001B3ull;
        }
    }
    for (uint32_t q0 = 16; q0 < nl; q0 += 16) {
        uint8_t v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = q0 + j < nl ? nm[q0 + j] : 0;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (q0 + j < nl) {
                h ^= v[j];
                h *= 0x100000001B3ull;
            }
        }
    }
    h = d_mix64(h);
    h = h ? h : 1ull;
    *h_out = h;
    uint32_t slot = (uint32_t)h & a.d_mask;
    uint64_t k;
    uint32_t id, dl;
    u32x4 n16;
    for (uint32_t step = 0;; ++step) {
        k = a.d_key[slot];
        id = a.d_id[slot];
        dl = a.d_len[slot];
        n16 = *(const u32x4*)(a.d_name16 + 16ull * slot);
        if (k == h) break;
        if (k == kEmpty || step >= a.d_mask) return false;
        slot = (slot + 1) & a.d_mask;
    }
    if (id == kNoId || id >= a.max_services || dl != nl) return false;
    bool eq = true;
#pragma unroll
    for (int j = 0; j < 16; ++j) eq &= (uint32_t)u[j] == ((n16[j >> 2] >> (8 * (j & 3))) & 0xFFu);  // (zero padded)
    if (!eq) return false;
    if (nl > 16) {
        const uint8_t* y = (const uint8_t*)(uintptr_t)a.d_ptr[slot];
        for (uint32_t q0 = 16; q0 < nl; q0 += 16) {
            uint8_t x[16], v[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                x[j] = q0 + j < nl ? nm[q0 + j] : 0;
                v[j] = q0 + j < nl ? y[q0 + j] : 0;
            }
            bool e2 = true;
#pragma unroll
            for (int j = 0; j < 16; ++j) e2 &= x[j] == v[j];
            if (!e2) return false;
        }
    }
    *id_out = id;
    return true;
}

__device__ __forceinline__ bool resolve16(const IngArgs& a, uint64_t i, const uint8_t* nm, uint32_t nl, uint64_t* h_out) {
    uint32_t id;
    if (!resolve16_id(a, nm, nl, h_out, &id)) return false;
    a.svc[i] = id;
    return true;
}

__device__ __forceinline__ void publish_name_h(const IngArgs& a, uint64_t i, const uint8_t* nm, uint32_t nl, uint64_t h) {
    a.svc_hash[i] = h;
    a.name_ptr[i] = (uint64_t)(uintptr_t)nm;
    a.name_len[i] = nl;
#if ZK_ING_LISTS
    list_add(a.pub, a.pub_n, i);
#endif
}

// ---- the span indexer's items (zk_ingest_dev_spans_items) ---------------------------------------
// CassieSpanStore.scala:214-242 as the host decoder restates it (zk_ingest.cpp, "indexer items"):
// only a span with an annotation is indexed; one key-value item per binary annotation with a host
// (that host's service, the key's hash); one annotation item per distinct non-core annotation value,
// from the group's minimum under Annotation.compare ((a.timestamp - b.timestamp).toInt, the first of
// equals kept, Annotation.scala:36-38), and only if that annotation has a host. Items are appended
// in any order (the sketches take a batch as a set). An item's service is resolved after D4: a host
// whose name is the fragment's own service refers to the fragment (kRefFrag), a name the dictionary
// holds resolves at once, a new one is published like a service name (kRefExtra: the extra list,
// which D3 / D4 run over as over fragments). A string whose hash is not in the captured set is
// copied out (scratch) and listed for the host, which keeps the hash -> string map.
// An attempt that runs out of scratch (or finds the set / extra list full) fails its fragment
// (kStNoScratch, decoded again after the host grows them); the items it appended stay, and
// skip_kv / skip_an tell the next attempt to pass over them (each kind is emitted in a fixed order).
constexpr uint32_t kRefFrag = 0x80000000u, kRefExtra = 0xC0000000u, kRefMask = 0x3FFFFFFFu;
// ZK_ING_ITEMS_DIAG (diagnostic builds only, results wrong): 1 = the items build without the item walk,
// 2 = the walk without emitting, 3 = emitting without the append
#ifndef ZK_ING_ITEMS_DIAG
#define ZK_ING_ITEMS_DIAG 0
#endif
constexpr uint32_t kUnknownLen = sizeof(kUnknown) - 1;

struct ItemState {
    uint32_t seen[2];  // this fragment's items handled so far ([0] key-value, [1] annotation)
    uint32_t skip[2];  // appended by an earlier attempt
    bool fail;
    uint64_t known[2];  // the lane's last string hash of each kind found in the set (0: none): the
                        // same key / value in the lane's next fragment skips the set probe
};

// 16 bytes of each side in flight at once (one round trip per 16 bytes, not one per byte)
__device__ __forceinline__ bool bytes_eq(const uint8_t* x, const uint8_t* y, uint32_t l) {
    for (uint32_t q0 = 0; q0 < l; q0 += 16) {
        uint8_t u[16], v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            u[j] = q0 + j < l ? x[q0 + j] : 0;
            v[j] = q0 + j < l ? y[q0 + j] : 0;
        }
        bool eq = true;
#pragma unroll
        for (int j = 0; j < 16; ++j) eq &= u[j] == v[j];
        if (!eq) return false;
    }
    return true;
}

// global bytes for a string the set or the dictionary keeps: g itself, else a scratch copy
__device__ __forceinline__ const uint8_t* global_copy(const IngArgs& a, const uint8_t* s, uint32_t l, const uint8_t* g) {
    if (g || l == 0) return g ? g : a.unknown;
    uint8_t* d = scratch_take(a, l);
    if (!d) return nullptr;
#pragma clang loop vectorize(disable)
    for (uint32_t q = 0; q < l; ++q) d[q] = s[q];
    return d;
}

// the key / value hash into the captured set (one probe when it is known); a probe run longer than
// kSetProbes counts as a full set (the host grows it: the set is kept at most half full between batches)
constexpr uint32_t kSetProbes = 256;
__device__ __forceinline__ bool capture_string(const IngArgs& a, uint64_t h, const uint8_t* s, uint32_t l, const uint8_t* g) {
    uint32_t slot = (uint32_t)h & a.s_mask;
    const uint8_t* ptr = nullptr;
    for (uint32_t step = 0; step < kSetProbes && step <= a.s_mask; ++step) {
        const uint64_t k = a.s_key[slot];
        if (k == h) return true;
        if (k == kEmpty) {
            if (!ptr && !(ptr = global_copy(a, s, l, g))) return false;  // scratch exhausted
            const unsigned long long old =
                atomicCAS((unsigned long long*)&a.s_key[slot], (unsigned long long)kEmpty, (unsigned long long)h);
            if (old == kEmpty) {
                const unsigned long long x = atomicAdd(&a.icnt[2], 1ull);  // < ns_cap: one entry per slot
                if (x < a.ns_cap) {
                    a.ns_hash[x] = h;
                    a.ns_ptr[x] = (uint64_t)(uintptr_t)ptr;
                    a.ns_len[x] = l;
                }
                return true;
            }
            if (old == h) return true;
        }
        slot = (slot + 1) & a.s_mask;
    }
    atomicAdd(&a.icnt[4], 1ull);  // the set is full
    return false;
}

// an item host's service (nm / nl: the effective name, g: its global bytes or null)
__device__ __forceinline__ bool item_service(const IngArgs& a, uint64_t i, const uint8_t* nm, uint32_t nl, const uint8_t* g,
                             const uint8_t* snm, uint32_t snl, bool snamed, uint32_t* enc) {
    if (snamed && nl == snl && bytes_eq(nm, snm, nl)) {
        *enc = kRefFrag | (uint32_t)i;
        return true;
    }
    uint64_t h;
    uint32_t id;
    if (resolve16_id(a, nm, nl, &h, &id)) {
        *enc = id;
        return true;
    }
    const uint8_t* ptr = global_copy(a, nm, nl, g);
    if (!ptr) return false;
    const unsigned long long x = atomicAdd(&a.icnt[3], 1ull);
    if (x >= a.x_cap) return false;  // the extra list is full (the host sees the count past x_cap)
    a.x_hash[x] = h;
    a.x_ptr[x] = (uint64_t)(uintptr_t)ptr;
    a.x_len[x] = nl;
    a.x_keep[x] = 1u;
    a.x_status[x] = kStOk;
    a.x_list[x] = (uint32_t)x;
    *enc = kRefExtra | (uint32_t)x;
    return true;
}

constexpr uint32_t kItemChunk = 512, kNoChunk = 0xFFFFFFFFu;

// ch (the LDS decoder): the wave's current chunk and its fill per kind, {c0, used0, c1, used1} in LDS;
// null (the global-memory decoder): one atomic per wave-append on the direct counters
__device__ __forceinline__ void item_append(const IngArgs& a, uint32_t kind, uint32_t enc, uint64_t h, uint32_t* ch) {
    if (ch) {
        const unsigned long long m = __ballot(1);
        const uint32_t ln = __lane_id();
        const uint32_t ld = (uint32_t)__ffsll(m) - 1u;
        const uint32_t cnt = (uint32_t)__popcll(m), r = (uint32_t)__popcll(m & ((1ull << ln) - 1ull));
        const uint32_t c = ch[2 * kind], used = ch[2 * kind + 1];
        uint32_t pc, pj;
        if (used + cnt <= kItemChunk) {
            pc = c;
            pj = used + r;
            if (ln == ld) ch[2 * kind + 1] = used + cnt;
        } else {
            uint32_t nc = 0;
            if (ln == ld) {
                nc = (uint32_t)atomicAdd(&a.icnt[11 + kind], 1ull);
                if (c < a.ck_cap) a.ck_fill[kind][c] = kItemChunk;  // (c is full now)
            }
            nc = (uint32_t)__shfl((int)nc, (int)ld);
            const uint32_t room = kItemChunk - used;
            pc = r < room ? c : nc;
            pj = r < room ? used + r : r - room;
            if (ln == ld) {
                ch[2 * kind] = nc;
                ch[2 * kind + 1] = cnt - room;
            }
        }
        if (pc < a.ck_cap) {
            const uint64_t q = (uint64_t)pc * kItemChunk + pj;
            a.ck_svc[kind][q] = enc;
            a.ck_key[kind][q] = h;
        } else {
            atomicAdd(&a.icnt[7 + kind], 1ull);
        }
        return;
    }
    const unsigned long long mask = __ballot(1);
    const uint32_t lane = __lane_id();
    const uint32_t leader = (uint32_t)__ffsll(mask) - 1u;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(&a.icnt[kind], (unsigned long long)__popcll(mask));
    base = __shfl(base, (int)leader);
    const uint64_t pos = base + (uint64_t)__popcll(mask & ((1ull << lane) - 1ull));
    if (kind == 0) {
        if (pos < a.kv_cap) {
            a.kv_svc[pos] = enc;
            a.kv_key[pos] = h;
        }
    } else if (pos < a.an_cap) {
        a.an_svc[pos] = enc;
        a.an_val[pos] = h;
    }
}

// one item: its host's name (hl == 0: absent or "", i.e. kUnknown), its key / value string, and the
// global copies of both (null: in LDS only); snm / snl / snamed: the fragment's own service
__device__ __forceinline__ void item_emit(const IngArgs& a, uint64_t i, ItemState& st, uint32_t kind, const uint8_t* hn, uint32_t hl,
                          const uint8_t* hg, const uint8_t* s, uint32_t sl, const uint8_t* sg, const uint8_t* snm,
                          uint32_t snl, bool snamed, uint32_t* ch) {
    if (st.fail || ZK_ING_ITEMS_DIAG == 2) return;
    if (st.seen[kind] < st.skip[kind]) {
        ++st.seen[kind];
        return;
    }
    if (hl == 0) {
        hn = a.unknown;
        hg = a.unknown;
        hl = kUnknownLen;
    }
    const uint64_t h = d_hash(s, sl);
    uint32_t enc;
    if ((h != st.known[kind] && !capture_string(a, h, s, sl, sg)) ||
        !item_service(a, i, hn, hl, hg, snm, snl, snamed, &enc)) {
        st.fail = true;
        return;
    }
    st.known[kind] = h;
    if (ZK_ING_ITEMS_DIAG == 3) {
        if (enc == 0x12345u) a.icnt[6] = h;  // (keeps the work)
    } else
        item_append(a, kind, enc, h, ch);
    ++st.seen[kind];
}

// -- the canonical layout (parse_record_fast accepted the span; lay: its list offsets and counts) --
struct FAnn {
    int64_t ts;
    uint32_t next, voff, vl, vc, hoff, hl;
    bool host;
};
__device__ __forceinline__ void fast_ann(const lds_u8* base, uint32_t p, FAnn& A) {
    LWin<6> c;  // [0A 0001] timestamp [0B 0002] value
    c.load(base, p);
    A.ts = (int64_t)c.be64<3>();
    A.vl = c.be32<14>();
    A.vc = c.raw32<18>() & 0xFFFFu;
    A.voff = p + 18u;
    const uint32_t q = p + 18u + A.vl;
    LWin<6> h;  // STOP, or [0C 0003] {[08 0001] ipv4 [06 0002] port [0B 0003] service_name} STOP STOP
    h.load(base, q);
    A.host = h.u8<0>() != T_STOP;
    A.hl = A.host ? h.be32<18>() : 0u;
    A.hoff = q + 22u;
    A.next = A.host ? q + 24u + A.hl : q + 1u;
}
__device__ __forceinline__ bool fast_core(const FAnn& A) {
    const uint32_t c0 = A.vc & 0xFFu, c1 = A.vc >> 8;
    return A.vl == 2u && ((c0 == 'c' && (c1 == 's' || c1 == 'r')) || (c0 == 's' && (c1 == 'r' || c1 == 's')));
}

// gb: base as a generic pointer; gx: the global address of base offset 0 (0: the bytes are in LDS only)
__device__ __forceinline__ void items_fast(const IngArgs& a, uint64_t i, ItemState& st, const lds_u8* base, const uint32_t lay[4],
                           uintptr_t gx, const uint8_t* snm, uint32_t snl, bool snamed, uint32_t* ch) {
    if (lay[1] == 0u || ZK_ING_ITEMS_DIAG == 1) return;  // not indexed (CassieSpanStore.scala:214-218)
    const uint8_t* gb = (const uint8_t*)base;
    auto G = [&](uint32_t off) -> const uint8_t* { return gx ? (const uint8_t*)(gx + off) : nullptr; };
    uint32_t p = lay[0];
    for (uint32_t k = 0; k < lay[1] && !st.fail; ++k) {
        FAnn A;
        fast_ann(base, p, A);
        if (!fast_core(A)) {
            bool rep = true;  // the first of its value?
            uint32_t q = lay[0];
            for (uint32_t j = 0; j < k; ++j) {
                FAnn B;
                fast_ann(base, q, B);
                if (!fast_core(B) && B.vl == A.vl && bytes_eq(gb + B.voff, gb + A.voff, A.vl)) {
                    rep = false;
                    break;
                }
                q = B.next;
            }
            if (rep) {
                FAnn M = A;  // the group's minimum
                q = A.next;
                for (uint32_t j = k + 1; j < lay[1]; ++j) {
                    FAnn B;
                    fast_ann(base, q, B);
                    if (!fast_core(B) && B.vl == A.vl && (int32_t)(uint32_t)((uint64_t)M.ts - (uint64_t)B.ts) > 0 &&
                        bytes_eq(gb + B.voff, gb + A.voff, A.vl))
                        M = B;
                    q = B.next;
                }
                if (M.host)
                    item_emit(a, i, st, 1u, gb + M.hoff, M.hl, G(M.hoff), gb + A.voff, A.vl, G(A.voff), snm, snl, snamed, ch);
            }
        }
        p = A.next;
    }
    p = lay[2];
    for (uint32_t k = 0; k < lay[3] && !st.fail; ++k) {
        // [0B 0001] key [0B 0002] value [08 0003] annotation_type, then STOP or [0C 0004] endpoint STOP STOP
        LWin<2> k1;
        k1.load(base, p);
        const uint32_t kl = k1.be32<3>(), koff = p + 7u;
        LWin<2> k2;
        k2.load(base, koff + kl);
        const uint32_t p3 = koff + kl + 7u + k2.be32<3>();
        LWin<8> k3;
        k3.load(base, p3);
        const bool host = k3.u8<7>() != T_STOP;
        const uint32_t hl = host ? k3.be32<25>() : 0u, hoff = p3 + 29u;
        if (host) item_emit(a, i, st, 0u, gb + hoff, hl, G(hoff), gb + koff, kl, G(koff), snm, snl, snamed, ch);
        p = host ? p3 + 31u + hl : p3 + 8u;
    }
}

// -- any layout (the generic walk accepted the span): the host decoder's read_span semantics --
template <class P>
struct GAnn {
    int64_t ts;
    P v;  // null: no value field
    uint32_t vl;
    bool host;
    P hn;  // null: the host has no service_name field
    uint32_t hl;
};
template <class P>
struct GBann {
    P k;
    uint32_t kl;
    bool host;
    P hn;
    uint32_t hl;
};
// the annotations (field 6 lists) or binary annotations (field 8 lists) of a span, in order
template <class P>
struct GItemIter {
    DRdT<P> r;
    int32_t left;
    int16_t list_id;
    __device__ bool next_elem() {  // positions r at the next element of a list_id list of structs
        for (;;) {
            if (left > 0) {
                --left;
                return true;
            }
            uint8_t t;
            int16_t fid;
            if (!r.field(&t, &fid)) return false;
            if (fid == list_id && t == T_LIST) {
                const uint8_t et = r.u8();
                const int32_t c = r.i32();
                if (!r.ok || c < 0) return false;
                if (et == T_STRUCT)
                    left = c;
                else
                    for (int32_t q = 0; r.ok && q < c; ++q) skip_flat(r, et);
            } else {
                skip_flat(r, t);
            }
            if (!r.ok) return false;
        }
    }
    __device__ bool next(GAnn<P>& A) {
        if (!next_elem()) return false;
        A.ts = 0;
        A.v = nullptr;
        A.vl = 0;
        A.host = false;
        A.hn = nullptr;
        A.hl = 0;
        for (;;) {
            uint8_t at;
            int16_t aid;
            if (!r.field(&at, &aid)) break;
            if (aid == 1 && at == T_I64)
                A.ts = r.i64();
            else if (aid == 2 && at == T_STRING)
                r.str(&A.v, &A.vl);
            else if (aid == 3 && at == T_STRUCT) {
                A.host = true;
                read_endpoint(r, &A.hn, &A.hl);
            } else
                skip_flat(r, at);
        }
        return r.ok;
    }
    __device__ bool next(GBann<P>& B) {
        if (!next_elem()) return false;
        B.k = nullptr;
        B.kl = 0;
        B.host = false;
        B.hn = nullptr;
        B.hl = 0;
        for (;;) {
            uint8_t bt;
            int16_t bid;
            if (!r.field(&bt, &bid)) break;
            if (bid == 1 && bt == T_STRING)
                r.str(&B.k, &B.kl);
            else if (bid == 4 && bt == T_STRUCT) {
                B.host = true;
                read_endpoint(r, &B.hn, &B.hl);
            } else
                skip_flat(r, bt);
        }
        return r.ok;
    }
};

template <class P>
__device__ __forceinline__ bool g_same_value(const GAnn<P>& A, const GAnn<P>& B) {
    if ((A.v == nullptr) != (B.v == nullptr) || A.vl != B.vl) return false;
    return A.v == nullptr || A.vl == 0 || bytes_eq((const uint8_t*)A.v, (const uint8_t*)B.v, A.vl);
}

// gsrc: the global address of src (null: src is in LDS only)
template <class P>
__device__ void items_generic(const IngArgs& a, uint64_t i, ItemState& st, P src, uint64_t len, const uint8_t* gsrc,
                              const uint8_t* snm, uint32_t snl, bool snamed, uint32_t* ch) {
    auto G = [&](P p) -> const uint8_t* { return gsrc ? gsrc + (p - src) : nullptr; };
    GItemIter<P> o{DRdT<P>{src, src + len, true}, 0, 6};
    GAnn<P> A, B;
    {
        GItemIter<P> z = o;
        if (!z.next(A)) return;  // no annotation: not indexed
    }
    int c;
    for (uint32_t k = 0; !st.fail && o.next(A); ++k) {
        if (is_core(A.v, A.vl, &c)) continue;
        bool rep = true;
        GItemIter<P> e{DRdT<P>{src, src + len, true}, 0, 6};
        for (uint32_t j = 0; j < k && e.next(B); ++j)
            if (!is_core(B.v, B.vl, &c) && g_same_value(A, B)) {
                rep = false;
                break;
            }
        if (!rep) continue;
        GAnn<P> M = A;
        GItemIter<P> l = o;
        while (l.next(B))
            if (!is_core(B.v, B.vl, &c) && g_same_value(A, B) &&
                (int32_t)(uint32_t)((uint64_t)M.ts - (uint64_t)B.ts) > 0)
                M = B;
        if (!M.host) continue;
        const bool hv = M.hn != nullptr && M.hl > 0;
        const bool vv = A.v != nullptr && A.vl > 0;
        item_emit(a, i, st, 1u, hv ? (const uint8_t*)M.hn : nullptr, hv ? M.hl : 0u, hv ? G(M.hn) : nullptr,
                  vv ? (const uint8_t*)A.v : a.unknown, vv ? A.vl : 0u, vv ? G(A.v) : a.unknown, snm, snl, snamed, ch);
    }
    GItemIter<P> b{DRdT<P>{src, src + len, true}, 0, 8};
    GBann<P> K;
    while (!st.fail && b.next(K)) {
        if (!K.host) continue;
        const bool hv = K.hn != nullptr && K.hl > 0;
        const bool kv = K.k != nullptr && K.kl > 0;
        item_emit(a, i, st, 0u, hv ? (const uint8_t*)K.hn : nullptr, hv ? K.hl : 0u, hv ? G(K.hn) : nullptr,
                  kv ? (const uint8_t*)K.k : a.unknown, kv ? K.kl : 0u, kv ? G(K.k) : a.unknown, snm, snl, snamed, ch);
    }
}

__device__ __forceinline__ void items_failed(const IngArgs& a, uint64_t i, const ItemState& st) {
    a.status[i] = kStNoScratch;
    a.skip_kv[i] = st.seen[0];
    a.skip_an[i] = st.seen[1];
}

// D2 (global memory): a fragment marked `mode` (kStDefer by the LDS kernel, or kStNoScratch)
template <bool kItems>
__device__ __forceinline__ void ing_decode_one(const IngArgs& a, uint64_t i, uint32_t mode) {
    if (a.status[i] != mode) return;
    a.status[i] = kStOk;
    a.keep[i] = 0u;
    a.svc_hash[i] = 0ull;
    const uint64_t b = a.offsets[i], e = a.ends[i];
    const uint8_t* src = a.buf + b;
    uint64_t len = e - b;
    if (a.snappy) {
        uint32_t h[5];
        uint64_t raw;
        head_bytes(a, true, b, e, h);
        if (head_status(true, b, e, h, &raw) != kStOk) {  // (checked before it was deferred)
            a.status[i] = kStUndecodable;
            return;
        }
        uint8_t* dst = scratch_take(a, raw);
        if (!dst) {
            a.status[i] = kStNoScratch;
            return;
        }
        if (!snappy_block(src, len, dst, raw)) {
            a.status[i] = kStUndecodable;
            return;
        }
        src = dst;
        len = raw;
    }
    const uint8_t* nm;
    uint32_t nl;
    const int r = parse_record(a, i, src, len, &nm, &nl);
    if (r < 0) return;
    if (r) publish_name(a, i, nm, nl);
    if constexpr (kItems) {  // a deferred fragment's first attempt (skips 0), or a failed one's next
        ItemState st{{0u, 0u}, {a.skip_kv[i], a.skip_an[i]}, false, {0ull, 0ull}};
        items_generic(a, i, st, src, len, src, nm, nl, r == 1, nullptr);
        if (st.fail) {
            items_failed(a, i, st);
            return;
        }
    }
    a.keep[i] = 1u;
}

// the deferred fragments (the LDS decoder's list), or every fragment marked kStNoScratch
// kItems: the items build of the decoders (zk_ingest_dev_spans_items), compiled apart so that the
// records-only kernels keep their registers
template <bool kItems>
__global__ __launch_bounds__(kIngWG) void k_ing_decode(IngArgs a, uint32_t mode) {
    if (mode == kStDefer) {
        ING_FOR_LIST(a.def, a.def_n, i) ing_decode_one<kItems>(a, i, mode);
    } else {
        for (uint64_t i = (uint64_t)blockIdx.x * kIngWG + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * kIngWG)
            ing_decode_one<kItems>(a, i, mode);
    }
}

// D2 (LDS): one wave per block of a.lds_block consecutive fragments, in rounds. A round takes the
// next fragments (at most 64, one per lane) whose LDS regions fit the wave's kLdsBudget bytes. A
// lane's region holds its decompressed Span at the front and its compressed bytes at the back
// (copied in with aligned 16-B loads): Snappy decompresses in place, front to back, and a step
// that would write over input not yet read defers the fragment instead (checked per element, so it
// never corrupts). The Span is then parsed from LDS (every dependent byte read is an LDS round trip
// instead of an L1/L2 one). At 20 KiB per wave, 8 waves fit a CU (separate in/out buffers for 64
// fragments needed 40 KiB: one wave per SIMD). Deferred fragments (a region larger than the budget,
// or an unsafe in-place step) go to the global-memory kernel. Service names are copied out to the
// global scratch (the dictionary kernels read them after this kernel).
constexpr uint32_t kLdsWG = 64;
#ifndef ZK_ING_BUDGET
#define ZK_ING_BUDGET 20480  // LDS bytes per wave (8 waves per CU)
#endif
constexpr uint32_t kLdsBudget = ZK_ING_BUDGET;
// ZK_ING_TAIL: 1 = a region keeps 16 bytes after its input for the copy-in's last 16-byte block;
// 0 = that block may spill up to 15 bytes into the next region's first bytes (output the next
// lane writes before it reads them), with 16 bytes kept free at the end of the wave's buffer.
// ZK_ING_SKEW: 1 = a lane's Span starts 4 * (lane group) bytes into its region (bank spread).
#ifndef ZK_ING_TAIL
#define ZK_ING_TAIL 1
#endif
#ifndef ZK_ING_SKEW
#define ZK_ING_SKEW 0  // off since round 5: 4.70 -> 4.65 ms (profiles/r05/ab_ingest_layout.txt)
#endif
constexpr uint32_t kLdsUse = kLdsBudget - (ZK_ING_TAIL ? 0u : 16u);  // bytes the regions may take
constexpr uint32_t kLdsBlock = 1024;  // fragments per wave for large batches; smaller batches take
                                      // smaller blocks (lds_block_for) so that they still fill the GPU
// Region bytes beyond max(raw, compressed): the input's placement (16 B of block tail + up to 15 of
// misalignment) and the lane's bank skew (up to 12). A region of raw + slack bytes also holds the
// output's final lead over the input (raw - compressed); a Snappy stream whose lead is larger part
// way through is caught by the in-place check and deferred. 48 (was 80): 55 lanes per round instead
// of 51 on the bench's fragments, 6.47 -> 5.97 ms (profiles/r05/ab_ingest_slack.txt).
#ifndef ZK_ING_SLACK
#define ZK_ING_SLACK 48
#endif
constexpr uint32_t kLdsSlack = ZK_ING_SLACK;
constexpr uint32_t kLdsUniformCap = 640;  // largest region (bytes) of a uniform round

// Snappy block from in = out + D (the same region), in place: false with *unsafe set when a step
// would write over input bytes not yet read. ZK_ING_OVERCOPY: a literal or a copy (offset >= 8)
// runs as whole 8-byte steps when the output trails the unread input by 8 bytes or more, instead
// of 8-byte steps and a byte loop for the rest (each byte a dependent LDS read and write).
#ifndef ZK_ING_OVERCOPY
#define ZK_ING_OVERCOPY 1
#endif
__device__ __forceinline__ bool snappy_inplace(lds_u8* out, uint64_t D, uint64_t n, uint64_t len, bool* unsafe) {
    const lds_u8* in = out + D;
    uint64_t dl, hdr;
    if (!snappy_hdr(in, n, &dl, &hdr) || dl != len) return false;
    uint64_t o = 0, i = hdr;
    while (i < n) {
        const uint8_t tag = in[i++];
        uint64_t l, off;
        const uint32_t kind = tag & 3;
        if (kind == 0) {
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
            // an 8-byte step writes output [o + k, o + k + 8) after reading input [i + k, i + k + 8):
            // it never reaches unread input while o <= D + i
            if (o > D + i) {
                *unsafe = true;
                return false;
            }
            uint64_t k = 0;
#if ZK_ING_OVERCOPY
            if (o + 8 <= D + i) {  // whole 8-byte steps: the last writes < 8 bytes past the literal, over
                                   // input already read or output the next tags write again
                for (; k < l; k += 8) cp8(out + o + k, in + i + k);
                i += l;
                o += l;
                continue;
            }
#endif
            for (; k + 8 <= l; k += 8) cp8(out + o + k, in + i + k);
            #pragma clang loop vectorize(disable)  // (a vectorised byte loop reads LDS with unaligned ds_read_b128)
            for (; k < l; ++k) out[o + k] = in[i + k];
            i += l;
            o += l;
            continue;
        }
        if (kind == 1) {
            if (i + 1 > n) return false;
            l = ((tag >> 2) & 7) + 4;
            off = ((uint64_t)(tag >> 5) << 8) | in[i];
            i += 1;
        } else if (kind == 2) {
            if (i + 2 > n) return false;
            l = (tag >> 2) + 1;
            off = (uint64_t)in[i] | ((uint64_t)in[i + 1] << 8);
            i += 2;
        } else {
            if (i + 4 > n) return false;
            l = (tag >> 2) + 1;
            off = (uint64_t)in[i] | ((uint64_t)in[i + 1] << 8) | ((uint64_t)in[i + 2] << 16) |
                  ((uint64_t)in[i + 3] << 24);
            i += 4;
        }
        if (off == 0 || off > o || o + l > len) return false;
        if (o + l > D + i) {  // the copy would reach the next unread input byte
            *unsafe = true;
            return false;
        }
#if ZK_ING_OVERCOPY
        if (off >= 8 && o + l + 8 <= D + i) {  // whole 8-byte steps (each reads bytes already written)
            for (uint64_t k = 0; k < l; k += 8) cp8(out + o + k, out + o - off + k);
            o += l;
            continue;
        }
#endif
        backref_copy(out, o, off, l);
        o += l;
    }
    return o == len;
}

#ifndef ZK_ING_SNAPPY_PIPE
#define ZK_ING_SNAPPY_PIPE 1
#endif
__device__ __forceinline__ void st8(lds_u8* d, uint64_t v) {
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = (uint8_t)(v >> (8 * k));
}

// snappy_inplace with one dependent LDS round trip per tag instead of up to three (tag, then its
// parameter bytes, then the source): a tag and its parameters come from an 8-byte window read
// while the previous tag's copy was in flight, and a copy's source is read 16 bytes at a time
// before its stores. The window lies at or past in + i, above every byte the tag's copy writes
// (the in-place checks below), so reading it first is safe. Same result, same failures, same
// unsafe verdicts as snappy_inplace.
__device__ __forceinline__ bool snappy_inplace_pipe(lds_u8* out, uint64_t D, uint64_t n, uint64_t len, bool* unsafe) {
    const lds_u8* in = out + D;
    uint64_t dl, hdr;
    if (!snappy_hdr(in, n, &dl, &hdr) || dl != len) return false;
    uint64_t o = 0, i = hdr;
    uint64_t w = ld_u64(in + i);  // in[i, i + 8): bytes past n are region bytes, used only after a bounds check
    while (i < n) {
        const uint32_t tag = (uint32_t)w & 0xFFu;
        const uint32_t kind = tag & 3u;
        uint64_t l, src, off = 0;  // src: the copy's source, as an offset from out
        bool whole8, pairs;
        if (kind == 0) {
            l = tag >> 2;
            uint64_t s = i + 1;
            if (l >= 60) {
                const uint32_t nb = (uint32_t)l - 59;
                if (s + nb > n) return false;
                l = (w >> 8) & (nb == 4 ? 0xFFFFFFFFull : ((1ull << (8 * nb)) - 1));
                s += nb;
            }
            l += 1;
            if (s + l > n || o + l > len) return false;
            if (o > D + s) {
                *unsafe = true;
                return false;
            }
            i = s + l;
            src = D + s;
            whole8 = o + 8 <= D + s;  // as snappy_inplace's overcopy condition
            pairs = true;             // the source lies above the stores
        } else {
            uint64_t adv;
            if (kind == 1) {
                adv = 2;
                l = ((tag >> 2) & 7) + 4;
                off = ((uint64_t)(tag >> 5) << 8) | ((w >> 8) & 0xFFu);
            } else if (kind == 2) {
                adv = 3;
                l = (tag >> 2) + 1;
                off = (w >> 8) & 0xFFFFu;
            } else {
                adv = 5;
                l = (tag >> 2) + 1;
                off = (w >> 8) & 0xFFFFFFFFull;
            }
            if (i + adv > n) return false;
            i += adv;
            if (off == 0 || off > o || o + l > len) return false;
            if (o + l > D + i) {
                *unsafe = true;
                return false;
            }
            src = o - off;
            whole8 = off >= 8 && o + l + 8 <= D + i;
            pairs = off >= 16;  // a 16-byte read never reaches this copy's own stores
        }
        const uint64_t wn = ld_u64(in + i);  // the next tag's window, ahead of this tag's stores
        if (whole8 && pairs) {
            for (uint64_t k = 0; k < l; k += 16) {
                const uint64_t v0 = ld_u64(out + src + k), v1 = ld_u64(out + src + k + 8);
                st8(out + o + k, v0);
                if (k + 8 < l) st8(out + o + k + 8, v1);
            }
        } else if (whole8) {
            for (uint64_t k = 0; k < l; k += 8) cp8(out + o + k, out + src + k);
        } else if (kind == 0) {
            uint64_t k = 0;
            for (; k + 8 <= l; k += 8) cp8(out + o + k, out + src + k);
            #pragma clang loop vectorize(disable)  // (a vectorised byte loop reads LDS with unaligned ds_read_b128)
            for (; k < l; ++k) out[o + k] = out[src + k];
        } else {
            backref_copy(out, o, off, l);
        }
        o += l;
        w = wn;
    }
    return o == len;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(v, d);
        if ((int)(threadIdx.x & 63) >= d) v += o;
    }
    return v;
}

// ---- diagnostic phase stamps (separate build with -DZK_ING_STAMPS; never in the product .so) --
#ifdef ZK_ING_STAMPS
__device__ unsigned long long g_ing_stamps[8];
__device__ __forceinline__ unsigned long long ing_memtime() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
#define ING_STAMP_DECL                            \
    unsigned long long ing_prev = ing_memtime();  \
    unsigned long long ing_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define ING_STAMP(k)                                      \
    do {                                                  \
        const unsigned long long ing_t = ing_memtime();   \
        ing_acc[k] += ing_t - ing_prev;                   \
        ing_prev = ing_t;                                 \
    } while (0)
#define ING_STAMP_FLUSH()                                                          \
    do {                                                                           \
        if (threadIdx.x == 0)                                                      \
            for (int q = 0; q < 8; ++q) atomicAdd(&g_ing_stamps[q], ing_acc[q]);  \
    } while (0)
#else
#define ING_STAMP_DECL
#define ING_STAMP(k)
#define ING_STAMP_FLUSH()
#endif

// ZK_ING_PREFETCH: the next round's fragments' first kPreBlk 16-byte blocks are loaded into
// registers during this round (with their headers), so a round's copy-in waits on no global load
// for fragments of up to kPreBlk * 16 - 15 bytes.
#ifndef ZK_ING_PREFETCH
#define ZK_ING_PREFETCH 1
#endif
constexpr int kPreBlk = 16;
typedef unsigned int ing_u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) ing_u32x4 ing_g_u32x4;

__device__ __forceinline__ uint32_t copy_blocks(const uint8_t* buf, uint64_t b, uint64_t e, bool h, ing_g_u32x4** g) {
    const uint32_t mis = (uint32_t)((uintptr_t)(buf + b) & 15u);
    *g = (ing_g_u32x4*)((uintptr_t)(buf + b) & ~(uintptr_t)15);
    return h && e > b ? (uint32_t)((e - b + mis + 15) >> 4) : 0u;
}

template <bool kItems>
__global__ __launch_bounds__(kLdsWG) void k_ing_decode_lds(IngArgs a) {
    constexpr bool kPre = ZK_ING_PREFETCH && !kItems;  // (the items build has no registers for it)
    uint64_t known[2] = {0ull, 0ull};  // items: the lane's last string hashes found in the set
    __shared__ __align__(16) uint8_t s_buf[kLdsBudget];
    // items: the wave's item chunks ({chunk, used} per kind) in the last 16 bytes (the regions keep off)
    constexpr uint32_t kUse = kItems ? kLdsUse - 16u : kLdsUse;
    uint32_t* const ch = kItems ? (uint32_t*)(s_buf + kLdsBudget - 16u) : nullptr;
    const uint32_t lane = threadIdx.x;
    if constexpr (kItems) {
        if (lane < 4) ch[lane] = (lane & 1u) ? kItemChunk : kNoChunk;  // no chunk yet: the first append takes one
    }
    const uint64_t blk0 = (uint64_t)blockIdx.x * a.lds_block;
    const uint64_t blk1 = blk0 + a.lds_block < a.n ? blk0 + a.lds_block : a.n;
    ING_STAMP_DECL
    // a round's fragment extents and Snappy headers are loaded during the round before (the first
    // round's here), so no round starts with a dependent global round trip
    bool nh = blk0 + lane < blk1;
    uint64_t nb = nh ? a.offsets[blk0 + lane] : 0, ne = nh ? a.ends[blk0 + lane] : 0;
    uint32_t hb[5];
    head_bytes(a, nh, nb, ne, hb);
    ing_u32x4 pre[kPreBlk];
    if constexpr (kPre) {
        ing_g_u32x4* pg;
        const uint32_t pn = copy_blocks(a.buf, nb, ne, nh, &pg);
#pragma unroll
        for (int c = 0; c < kPreBlk; ++c)
            if ((uint32_t)c < pn) pre[c] = pg[c];
    }
    for (uint64_t f0 = blk0; f0 < blk1;) {  // uniform
        const uint64_t i = f0 + lane;
        const bool have = i < blk1;
        const uint64_t b = nb;
        uint64_t clen = 0, raw = 0;
        uint32_t need = 0;
        uint8_t st = kStInvalid;
        if (have) {
            st = head_status(a.snappy, nb, ne, hb, &raw);
            if (st == kStOk) {
                clen = ne - nb;
                const uint64_t r = ((raw > clen ? raw : clen) + kLdsSlack + 15) & ~15ull;
                need = r > kUse ? kUse + 1 : (uint32_t)r;
            }
        }
        // Uniform layout (every region of the round has the size R of the largest, R / 16 odd, lane
        // L at L * R with a skew of 4 * (L / 16) bytes): lanes parsing the same field offset then
        // hit 64 different banks, where regions packed back to back at sizes that are multiples of
        // 16 B put several lanes on one bank. Used while no region of the next 64 exceeds
        // kLdsUniformCap; else regions are packed.
        uint32_t mx = need;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const uint32_t y = (uint32_t)__shfl_xor((int)mx, o);
            mx = y > mx ? y : mx;
        }
        const bool uniform = mx <= kLdsUniformCap;
        uint32_t R = need, R0, k;
        bool fits;
        if (uniform) {
            R = mx < 16u ? 16u : mx;
            if (((R >> 4) & 1u) == 0u) R += 16u;
            k = kUse / R;
            if (k > 64u) k = 64u;
            R0 = lane * R;
            fits = true;
        } else {
            const uint32_t incl = wave_incl_scan(need);
            // this round: the longest prefix of lanes that fits (at least lane 0, to make progress)
            k = (uint32_t)__popcll(__ballot(have && incl <= kUse));
            if (k == 0) k = 1;  // lane 0 alone does not fit: deferred below
            R0 = incl - need;
            fits = incl <= kUse;
        }
        ING_STAMP(0);
        // the next round's extents (its copy-in below waits for them in passing: loads return in order)
        nh = f0 + k + lane < blk1;
        nb = nh ? a.offsets[f0 + k + lane] : 0;
        ne = nh ? a.ends[f0 + k + lane] : 0;
        const bool go = lane < k && have && st == kStOk && fits;
        uint32_t D = 0, mis = 0;
        uint8_t* reg = s_buf + R0;
        if (lane < k && have) {
            a.keep[i] = 0u;
            a.svc_hash[i] = 0ull;
            if constexpr (kItems) {
                a.skip_kv[i] = 0u;
                a.skip_an[i] = 0u;
            }
            a.status[i] = st == kStOk && !fits ? kStDefer : st;
#if ZK_ING_LISTS
            if (st == kStOk && !fits) list_add(a.def, a.def_n, i);
#endif
            if (go) {
                mis = (uint32_t)((uintptr_t)(a.buf + b) & 15u);
                // input at offset D of the region (D = mis mod 16): its aligned 16-B blocks cover
                // [D - mis, D + clen + 15] inside [0, R) since R >= clen + kLdsSlack
                D = ((R - (ZK_ING_TAIL ? 16u : 0u) - (uint32_t)clen - mis) & ~15u) + mis;
                // 16-B blocks through a global-space pointer (global_load, not a flat load)
                ing_g_u32x4* g = (ing_g_u32x4*)((uintptr_t)(a.buf + b) & ~(uintptr_t)15);
                const uint32_t nblk = (uint32_t)((clen + mis + 15) >> 4);
                ing_u32x4* dst = reinterpret_cast<ing_u32x4*>(reg + D - mis);
                if constexpr (kPre) {
#pragma unroll
                    for (int c = 0; c < kPreBlk; ++c)
                        if ((uint32_t)c < nblk) dst[c] = pre[c];
                    for (uint32_t c = kPreBlk; c < nblk; ++c) dst[c] = g[c];
                } else {
                    for (uint32_t c = 0; c < nblk; ++c) dst[c] = g[c];
                }
            }
        }
        head_bytes(a, nh, nb, ne, hb);  // the next round's headers, in flight during this round's decode
        if constexpr (kPre) {
            ing_g_u32x4* pg;
            const uint32_t pn = copy_blocks(a.buf, nb, ne, nh, &pg);
#pragma unroll
            for (int c = 0; c < kPreBlk; ++c)
                if ((uint32_t)c < pn) pre[c] = pg[c];
        }
        if (go) {
            ING_STAMP(1);
            // the region as an LDS pointer: the decoder's byte and word reads become ds_read_*.
            // Regions start on 16-byte boundaries, i.e. on one of 8 bank offsets of a 32-bank
            // group; lanes parsing the same field at the same offset then collide. The
            // decompressed span starts 4 * (lane % 4) bytes in, spreading the lanes over all 32.
            lds_u8* const lreg = (lds_u8*)reg;
            const uint32_t skew = ZK_ING_SKEW ? 4u * (uniform ? (lane >> 4) & 3u : lane & 3u) : 0u;
            const lds_u8* src = lreg + D;
            uint64_t len = clen;
            bool ok = true, unsafe = false;
            if (a.snappy) {
#if ZK_ING_SNAPPY_PIPE
                ok = snappy_inplace_pipe(lreg + skew, D - skew, clen, raw, &unsafe);
#else
                ok = snappy_inplace(lreg + skew, D - skew, clen, raw, &unsafe);
#endif
                src = lreg + skew;
                len = raw;
            }
            ING_STAMP(2);
            if (!ok) {
                a.status[i] = unsafe ? kStDefer : kStUndecodable;
#if ZK_ING_LISTS
                if (unsafe) list_add(a.def, a.def_n, i);
#endif
            } else {
                const lds_u8* const lbase = (const lds_u8*)s_buf;
                const uint32_t p0 = (uint32_t)(src - lbase);
                uint32_t nmo, nl, lay[4];
                int r = parse_record_fast(a, i, lbase, p0, (uint32_t)len, &nmo, &nl, lay);
                const bool fast = r != -3;
                if (r == -3) {  // not the canonical layout: the generic walk
                    const uint8_t* gnm = nullptr;
                    r = parse_record(a, i, src, len, &gnm, &nl);
                    nmo = (r == 1 && gnm != (const uint8_t*)a.unknown) ? (uint32_t)(gnm - (const uint8_t*)lbase)
                                                                       : ~0u;
                }
                const bool unknown = nmo == ~0u;
                const uint8_t* nm = unknown ? a.unknown : (const uint8_t*)(lbase + nmo);
                if (unknown) nl = sizeof(kUnknown) - 1;
                ING_STAMP(3);
                if (r >= 0) {
#if ZK_ING_NAME16
                    uint64_t nh = 0;
                    if (r && !resolve16(a, i, nm, nl, &nh)) {
#else
                    if (r && !try_resolve(a, i, nm, nl, d_hash(nm, nl))) {
#endif
                        if (!unknown) {  // the name lies in this lane's own bytes
                            const uint64_t off = nmo - p0;
                            if (a.snappy) {
                                uint8_t* gd = scratch_take(a, nl);  // copy out to the scratch
                                if (gd) {
#pragma clang loop vectorize(disable)
                                    for (uint32_t q = 0; q < nl; ++q) gd[q] = nm[q];
                                } else {
                                    a.status[i] = kStNoScratch;
                                    r = -1;
                                }
                                nm = gd;
                            } else {
                                nm = a.buf + b + off;  // thrift codec: the name is in the input buffer
                            }
                        }
#if ZK_ING_NAME16
                        if (r >= 0) publish_name_h(a, i, nm, nl, nh);
#else
                        if (r >= 0) publish_name(a, i, nm, nl);
#endif
                    }
                    if (kItems && r >= 0) {
                        // the global address of LDS offset 0 (thrift codec: the input buffer)
                        const uintptr_t gx = a.snappy ? 0 : (uintptr_t)(a.buf + b) - p0;
                        ItemState st{{0u, 0u}, {0u, 0u}, false, {known[0], known[1]}};
                        if (fast)
                            items_fast(a, i, st, lbase, lay, gx, nm, nl, r == 1, ch);
                        else
                            items_generic(a, i, st, src, len, gx ? (const uint8_t*)(gx + p0) : nullptr, nm, nl, r == 1,
                                          ch);
                        known[0] = st.known[0];
                        known[1] = st.known[1];
                        if (st.fail) {
                            items_failed(a, i, st);
                            r = -1;
                        }
                    }
                    if (r >= 0) a.keep[i] = 1u;
                }
            }
        }
        ING_STAMP(4);
        f0 += k;
        __syncthreads();  // one wave: this round's LDS accesses complete before the next round's copies
        ING_STAMP(5);
    }
    if constexpr (kItems) {  // the fill of the wave's last chunk of each kind
        if (lane < 2) {
            const uint32_t c = ch[2 * lane];
            if (c < a.ck_cap) a.ck_fill[lane][c] = ch[2 * lane + 1];
        }
    }
    ING_STAMP_FLUSH();
}

__device__ __forceinline__ void ing_insert_one(const IngArgs& a, uint64_t i) {
    if (!a.keep[i]) return;
    const uint64_t h = a.svc_hash[i];
    if (!h) return;
    uint32_t slot = (uint32_t)h & a.d_mask;
    for (uint32_t step = 0; step <= a.d_mask; ++step) {
        const uint64_t seen = a.d_key[slot];  // read first: after the first batches every name is there
        if (seen == h) return;
        if (seen != kEmpty) {
            slot = (slot + 1) & a.d_mask;
            continue;
        }
        const unsigned long long old = atomicCAS((unsigned long long*)&a.d_key[slot], (unsigned long long)kEmpty,
                                                 (unsigned long long)h);
        if (old == kEmpty) {  // the first claimant names the slot (verified against the others in D4)
            a.d_ptr[slot] = a.name_ptr[i];
            a.d_len[slot] = a.name_len[i];
            atomicAdd(a.claims, 1ull);
            return;
        }
        if (old == h) return;
        slot = (slot + 1) & a.d_mask;
    }
}

__global__ __launch_bounds__(kIngWG) void k_ing_dict_insert(IngArgs a) {
    ING_FOR_LIST(a.pub, a.pub_n, i) ing_insert_one(a, i);
}

__device__ __forceinline__ void ing_lookup_one(const IngArgs& a, uint64_t i) {
    if (!a.keep[i]) return;
    const uint64_t h = a.svc_hash[i];
    if (!h) return;
    uint32_t slot = (uint32_t)h & a.d_mask;
    for (uint32_t step = 0; step <= a.d_mask; ++step) {
        const uint64_t k = a.d_key[slot];
        if (k == h) break;
        if (k == kEmpty) {
            slot = kNoId;
            break;
        }
        slot = (slot + 1) & a.d_mask;
    }
    if (slot == kNoId) {  // not in the table (a full table)
        a.status[i] = kStRange;
        a.keep[i] = 0u;
        return;
    }
    const uint32_t id = a.d_id[slot];
    if (id == kNoId) return;  // claimed in this batch, id not given yet: the host runs D4 again
    if (id >= a.max_services) {
        a.status[i] = kStRange;  // more distinct services than the decoder was sized for
        a.keep[i] = 0u;
        return;
    }
    // exact: the name bytes equal the slot's (a 64-bit hash collision is an error, not a merge)
    const uint8_t* x = (const uint8_t*)(uintptr_t)a.name_ptr[i];
    const uint8_t* y = (const uint8_t*)(uintptr_t)a.d_ptr[slot];
    const uint32_t l = a.name_len[i];
    bool same = l == a.d_len[slot];
    for (uint32_t q = 0; same && q < l; ++q) same = x[q] == y[q];
    if (!same) {
        a.status[i] = kStCollision;
        a.keep[i] = 0u;
        return;
    }
    a.svc[i] = id;
}

__global__ __launch_bounds__(kIngWG) void k_ing_lookup(IngArgs a) {
    ING_FOR_LIST(a.pub, a.pub_n, i) ing_lookup_one(a, i);
}

__global__ __launch_bounds__(kIngWG) void k_ing_compact(IngArgs a, zk_span_cols o) {
    const uint64_t i = (uint64_t)blockIdx.x * kIngWG + threadIdx.x;
    if (i >= a.n || !a.keep[i]) return;
    const uint32_t p = a.pos[i];
    ((uint64_t*)o.trace_id)[p] = a.tid[i];
    ((uint64_t*)o.span_id)[p] = a.sid[i];
    ((uint64_t*)o.parent_id)[p] = a.pid[i];
    ((int64_t*)o.first_ts)[p] = a.first[i];
    ((int64_t*)o.last_ts)[p] = a.last[i];
    ((uint32_t*)o.service_id)[p] = a.svc[i];
    ((uint32_t*)o.flags)[p] = a.flags[i];
}

// the names of a batch's new dictionary slots, gathered into the arena in one launch (from the
// scratch or the input buffer where D2 published them)
__global__ void k_ing_gather_names(const uint64_t* __restrict__ src, const uint64_t* __restrict__ dst_off,
                                   const uint32_t* __restrict__ len, uint32_t m, uint8_t* __restrict__ arena) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= m) return;
    const uint8_t* x = (const uint8_t*)(uintptr_t)src[k];
    uint8_t* y = arena + dst_off[k];
    for (uint32_t q = 0; q < len[k]; ++q) y[q] = x[q];
}

// Several stored batches as one (zk_ingest_dev_spans_multi): fragment i of the joined batch is
// fragment i - first[b] of batch b, where first[b] <= i < first[b + 1]; its extents relative to the
// lowest batch buffer (rel[b] = bufs[b] - base) go to starts / ends, so the decoder reads
// base + [starts[i], ends[i]) exactly as one batch's buf + [offsets[i], offsets[i + 1]).
struct IngMultiBatch {
    uint64_t rel;
    const uint64_t* offsets;
    uint64_t first;
};
__global__ void k_ing_multi_bounds(const IngMultiBatch* __restrict__ tab, uint32_t nb, uint64_t n,
                                   uint64_t* __restrict__ starts, uint64_t* __restrict__ ends) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t lo = 0, hi = nb;  // the last batch with first <= i (empty batches share a first)
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (tab[mid].first <= i)
            lo = mid;
        else
            hi = mid;
    }
    const IngMultiBatch t = tab[lo];
    const uint64_t j = i - t.first;
    starts[i] = t.rel + t.offsets[j];
    ends[i] = t.rel + t.offsets[j + 1];
}

__global__ void k_ing_count(const uint8_t* status, uint64_t n, unsigned long long* counts, unsigned int* first_bad) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t s = status[i];
    if (s == kStOk) return;
    atomicAdd(&counts[s], 1ull);
    atomicMin(first_bad, (unsigned int)(i < 0xFFFFFFFFull ? i : 0xFFFFFFFEull));
}

// the extra names' D4 failures: [5] collisions, [6] more services than max_services
// The extra names run through D3 / D4 as an IngArgs whose per-fragment arrays are the extra
// list's (x.n = its capacity: the count may have run past it in a failed attempt)
#define ING_FOR_EXTRA(x, i)                                                                        \
    const uint64_t ing_m = *(x).pub_n < (x).n ? *(x).pub_n : (x).n;                                \
    for (uint64_t ing_t = (uint64_t)blockIdx.x * kIngWG + threadIdx.x; ing_t < ing_m;             \
         ing_t += (uint64_t)gridDim.x * kIngWG)                                                   \
        if (const uint64_t i = (x).pub[ing_t]; true)

__global__ __launch_bounds__(kIngWG) void k_ing_dict_insert_x(IngArgs x) {
    ING_FOR_EXTRA(x, i) ing_insert_one(x, i);
}
__global__ __launch_bounds__(kIngWG) void k_ing_lookup_x(IngArgs x) {
    ING_FOR_EXTRA(x, i) ing_lookup_one(x, i);
}
__global__ __launch_bounds__(kIngWG) void k_ing_count_extra(IngArgs x) {
    ING_FOR_EXTRA(x, i) {
        const uint8_t s = x.status[i];
        if (s == kStCollision) atomicAdd(&x.icnt[5], 1ull);
        if (s == kStRange) atomicAdd(&x.icnt[6], 1ull);
    }
}

// item service references -> dictionary ids (after D4 of the fragments and the extra names; a.svc
// still holds the records at their fragment index)
__global__ __launch_bounds__(kIngWG) void k_ing_item_fixup(IngArgs a, uint64_t nkv, uint64_t nan) {
    for (uint64_t t = (uint64_t)blockIdx.x * kIngWG + threadIdx.x; t < nkv + nan; t += (uint64_t)gridDim.x * kIngWG) {
        uint32_t* sv = t < nkv ? &a.kv_svc[t] : &a.an_svc[t - nkv];
        const uint32_t v = *sv;
        if (v & kRefFrag) *sv = (v & (kRefExtra & ~kRefFrag)) ? a.x_svc[v & kRefMask] : a.svc[v & kRefMask];
    }
}

// The caller's item buffers of one kind: the LDS decoder's chunks (in chunk order, each chunk's fill;
// off = exclusive scan of the fills), then the global-memory decoder's direct items. [9 + kind] = the
// chunked items kept.
__global__ __launch_bounds__(kIngWG) void k_ing_item_compact(IngArgs a, uint32_t kind, uint32_t nch,
                                                             const uint32_t* __restrict__ off, uint64_t ndirect,
                                                             uint32_t* __restrict__ out_svc, uint64_t* __restrict__ out_key,
                                                             uint64_t cap) {
    const uint64_t F = nch ? (uint64_t)off[nch - 1] + a.ck_fill[kind][nch - 1] : 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) a.icnt[9 + kind] = F;
    const uint64_t nc = (uint64_t)nch * kItemChunk;
    const uint32_t* dsvc = kind ? a.an_svc : a.kv_svc;
    const uint64_t* dkey = kind ? a.an_val : a.kv_key;
    for (uint64_t t = (uint64_t)blockIdx.x * kIngWG + threadIdx.x; t < nc + ndirect; t += (uint64_t)gridDim.x * kIngWG) {
        uint64_t dst, src;
        const uint32_t* ss;
        const uint64_t* sk;
        if (t < nc) {
            const uint32_t c = (uint32_t)(t / kItemChunk), j = (uint32_t)(t % kItemChunk);
            if (j >= a.ck_fill[kind][c]) continue;
            dst = (uint64_t)off[c] + j;
            src = t;
            ss = a.ck_svc[kind];
            sk = a.ck_key[kind];
        } else {
            dst = F + (t - nc);
            src = t - nc;
            ss = dsvc;
            sk = dkey;
        }
        if (dst < cap) {
            out_svc[dst] = ss[src];
            out_key[dst] = sk[src];
        }
    }
}

// the captured-string set into a larger table (keys are distinct)
__global__ void k_ing_set_rehash(const uint64_t* __restrict__ old, uint64_t n_old, uint64_t* nw, uint32_t mask) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_old) return;
    const uint64_t k = old[t];
    if (k == kEmpty) return;
    uint32_t slot = (uint32_t)k & mask;
    while (atomicCAS((unsigned long long*)&nw[slot], (unsigned long long)kEmpty, (unsigned long long)k) != kEmpty)
        slot = (slot + 1) & mask;
}

}  // namespace
}  // namespace zk

using namespace zk;

struct zk_ingest_dev {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    uint32_t max_services = 0;
    uint32_t table = 0;
    // persistent dictionary
    uint64_t* d_key = nullptr;
    uint32_t* d_id = nullptr;
    uint64_t* d_ptr = nullptr;
    uint32_t* d_len = nullptr;
    uint8_t* d_name16 = nullptr;     // 16 bytes per slot: the first bytes of its name (zero padded)
    std::vector<uint8_t> name16;     // host mirror
    uint8_t* arena = nullptr;  // names, device copy (kUnknown first)
    uint64_t arena_cap = 0, arena_used = 0;
    std::vector<std::string> names;
    std::vector<uint32_t> slot_id;  // host mirror of d_id
    // per-batch scratch
    void* batch = nullptr;
    uint64_t batch_cap = 0;
    uint8_t* scratch = nullptr;  // Snappy: bump-allocated per batch (deferred Spans, new names)
    uint64_t scratch_cap = 0;
    uint64_t scratch_min = 0;    // first size (zk_ingest_dev_set_scratch; 0: from the batch size)
    void* cub = nullptr;
    size_t cub_cap = 0;
    unsigned long long* counts = nullptr;  // [8] per status, [8] first_bad, [10] scratch bytes taken,
                                           // [11] / [12] published / deferred list lengths, [13] claims,
                                           // [16..23) IngArgs::icnt (items)
    unsigned long long* h_counts = nullptr;  // pinned host copy of counts[0..23)
    // the span indexer's items (zk_ingest_dev_spans_items)
    uint64_t* s_key = nullptr;  // the captured-string set (hashes), open addressing
    uint32_t s_cap = 0;
    uint64_t s_count = 0;
    std::unordered_map<uint64_t, std::string> strings;  // hash -> the string first captured for it
    uint8_t* ns = nullptr;      // this batch's captured strings: hash u64 [s_cap], ptr u64, len u32
    uint64_t ns_cap = 0;
    uint8_t* xs = nullptr;      // extra names: hash, ptr u64; len, svc, keep, list u32; status u8 [x_cap]
    uint64_t x_cap = 0;
    uint8_t* istage = nullptr;  // item staging: the global decoder's direct items, the LDS decoder's chunks
    uint64_t istage_cap = 0;
    uint8_t* multi = nullptr;   // zk_ingest_dev_spans_multi: the batch table, then starts / ends [n]
    uint64_t multi_cap = 0;
    std::string err;
};

namespace {

zk_status dfail(zk_ingest_dev* g, zk_status s, const std::string& m) {
    if (g) g->err = m;
    return s;
}

#define ING_HIP(g, call)                                                                                \
    do {                                                                                                \
        hipError_t _e = (call);                                                                         \
        if (_e != hipSuccess)                                                                          \
            return dfail(g, is_refusal(_e) ? ZK_ERR_CAPACITY : ZK_ERR_HIP,                          \
                        std::string(#call) + ": " + launch_error_str(_e));                             \
    } while (0)

uint64_t align256(uint64_t x) { return (x + 255) & ~255ull; }

}  // namespace

extern "C" {

zk_status zk_ingest_dev_create(int32_t device, void* stream, uint32_t max_services, zk_ingest_dev** out) {
    ZK_GUARD_BEGIN
    if (!out || max_services == 0 || max_services > (1u << 20)) return ZK_ERR_INVALID_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0 || device < 0 || device >= ndev) return ZK_ERR_NO_DEVICE;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return ZK_ERR_NO_DEVICE;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return ZK_ERR_NO_DEVICE;
    zk_ingest_dev* g = new zk_ingest_dev();
    g->device = device;
    g->max_services = max_services;
    uint32_t t = 1024;
    while (t < 2 * max_services) t <<= 1;
    g->table = t;
    g->slot_id.assign(t, kNoId);
    g->name16.assign((size_t)t * 16, 0);
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) {
        if (stream) {
            g->stream = (hipStream_t)stream;
        } else {
            e = hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking);
            g->own_stream = true;
        }
    }
    g->arena_cap = 1 << 16;
    if (e == hipSuccess) e = hipMalloc(&g->d_key, (uint64_t)t * 8);
    if (e == hipSuccess) e = hipMalloc(&g->d_id, (uint64_t)t * 4);
    if (e == hipSuccess) e = hipMalloc(&g->d_ptr, (uint64_t)t * 8);
    if (e == hipSuccess) e = hipMalloc(&g->d_len, (uint64_t)t * 4);
    if (e == hipSuccess) e = hipMalloc(&g->d_name16, (uint64_t)t * 16);
    if (e == hipSuccess) e = hipMemsetAsync(g->d_name16, 0, (uint64_t)t * 16, g->stream);
    if (e == hipSuccess) e = hipMalloc(&g->arena, g->arena_cap);
    if (e == hipSuccess) e = hipMalloc(&g->counts, 32 * 8);
    if (e == hipSuccess) e = hipHostMalloc((void**)&g->h_counts, 32 * 8, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMemsetAsync(g->d_key, 0, (uint64_t)t * 8, g->stream);
    if (e == hipSuccess) e = hipMemsetAsync(g->d_id, 0xFF, (uint64_t)t * 4, g->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(g->arena, kUnknown, sizeof(kUnknown) - 1, hipMemcpyHostToDevice, g->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(g->stream);
    g->arena_used = sizeof(kUnknown) - 1;
    if (e != hipSuccess) {
        zk_ingest_dev_destroy(g);
        return ZK_ERR_HIP;
    }
    *out = g;
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_ingest_dev_destroy(zk_ingest_dev* g) {
    ZK_GUARD_BEGIN
    if (!g) return ZK_ERR_INVALID_ARG;
    hipSetDevice(g->device);
    if (g->stream) hipStreamSynchronize(g->stream);
    hipFree(g->d_key);
    hipFree(g->d_id);
    hipFree(g->d_ptr);
    hipFree(g->d_len);
    hipFree(g->d_name16);
    hipFree(g->arena);
    hipFree(g->counts);
    hipHostFree(g->h_counts);
    hipFree(g->batch);
    hipFree(g->scratch);
    hipFree(g->cub);
    hipFree(g->s_key);
    hipFree(g->ns);
    hipFree(g->xs);
    hipFree(g->istage);
    hipFree(g->multi);
    if (g->own_stream && g->stream) hipStreamDestroy(g->stream);
    delete g;
    return ZK_OK;
    ZK_GUARD_END
}

const char* zk_ingest_dev_last_error(const zk_ingest_dev* g) { return g ? g->err.c_str() : "null decoder"; }

zk_status zk_ingest_dev_set_scratch(zk_ingest_dev* g, uint64_t bytes) {
    ZK_GUARD_BEGIN
    if (!g) return ZK_ERR_INVALID_ARG;
    ING_HIP(g, hipSetDevice(g->device));
    ING_HIP(g, hipStreamSynchronize(g->stream));  // no batch may still use the old scratch
    hipFree(g->scratch);
    g->scratch = nullptr;
    g->scratch_cap = 0;
    g->scratch_min = bytes;  // allocated by the next Snappy batch
    return ZK_OK;
    ZK_GUARD_END
}

#ifdef ZK_ING_STAMPS
int zk_debug_ing_stamps(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_ing_stamps), 8 * 8) != hipSuccess) return 1;
    if (reset) {
        unsigned long long z[8] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_ing_stamps), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
#endif

}  // extern "C"

namespace {

// the captured-string set at a larger capacity (the caller holds the stream)
hipError_t grow_string_set(zk_ingest_dev* g, uint32_t cap) {
    uint64_t* nk = nullptr;
    hipError_t e = hipMalloc(&nk, (uint64_t)cap * 8);
    if (e == hipSuccess) e = hipMemsetAsync(nk, 0, (uint64_t)cap * 8, g->stream);
    if (e == hipSuccess && g->s_key)
        e = launch_checked("k_ing_set_rehash", k_ing_set_rehash, dim3((g->s_cap + 255) / 256), dim3(256), 0, g->stream,
                           (const uint64_t*)g->s_key, (uint64_t)g->s_cap, nk, cap - 1);
    if (e == hipSuccess) e = hipStreamSynchronize(g->stream);
    if (e != hipSuccess) {
        hipFree(nk);
        return e;
    }
    hipFree(g->s_key);
    g->s_key = nk;
    g->s_cap = cap;
    return hipSuccess;
}

// the list of captured strings (one entry per set slot at most), its first `keep` entries kept
hipError_t size_new_strings(zk_ingest_dev* g, uint64_t keep) {
    if (g->ns_cap >= g->s_cap) return hipSuccess;
    uint8_t* nn = nullptr;
    const uint64_t c = g->s_cap;
    hipError_t e = hipMalloc(&nn, c * 20);
    if (e == hipSuccess && keep) {
        e = hipMemcpyAsync(nn, g->ns, keep * 8, hipMemcpyDeviceToDevice, g->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(nn + c * 8, g->ns + g->ns_cap * 8, keep * 8, hipMemcpyDeviceToDevice, g->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(nn + c * 16, g->ns + g->ns_cap * 16, keep * 4, hipMemcpyDeviceToDevice, g->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(g->stream);
    if (e != hipSuccess) {
        hipFree(nn);
        return e;
    }
    hipFree(g->ns);
    g->ns = nn;
    g->ns_cap = c;
    return hipSuccess;
}

// the extra-name list at capacity c, its first `keep` entries kept
hipError_t size_extra(zk_ingest_dev* g, uint64_t c, uint64_t keep) {
    uint8_t* nx = nullptr;
    hipError_t e = hipMalloc(&nx, c * 33);
    const uint64_t o = g->x_cap;
    // layout: hash [c] u64, ptr [c] u64, len [c] u32, svc [c] u32, keep [c] u32, list [c] u32, status [c] u8
    const uint64_t off_new[7] = {0, c * 8, c * 16, c * 20, c * 24, c * 28, c * 32};
    const uint64_t off_old[7] = {0, o * 8, o * 16, o * 20, o * 24, o * 28, o * 32};
    const uint64_t w[7] = {8, 8, 4, 4, 4, 4, 1};
    for (int k = 0; k < 7 && e == hipSuccess && keep; ++k)
        e = hipMemcpyAsync(nx + off_new[k], g->xs + off_old[k], keep * w[k], hipMemcpyDeviceToDevice, g->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(g->stream);
    if (e != hipSuccess) {
        hipFree(nx);
        return e;
    }
    hipFree(g->xs);
    g->xs = nx;
    g->x_cap = c;
    return hipSuccess;
}

void bind_items(zk_ingest_dev* g, IngArgs& a, IngArgs& x) {
    a.s_key = g->s_key;
    a.s_mask = g->s_cap - 1;
    a.ns_hash = (uint64_t*)g->ns;
    a.ns_ptr = (uint64_t*)(g->ns + g->ns_cap * 8);
    a.ns_len = (uint32_t*)(g->ns + g->ns_cap * 16);
    a.ns_cap = g->ns_cap;
    const uint64_t c = g->x_cap;
    a.x_hash = (uint64_t*)g->xs;
    a.x_ptr = (uint64_t*)(g->xs + c * 8);
    a.x_len = (uint32_t*)(g->xs + c * 16);
    a.x_svc = (uint32_t*)(g->xs + c * 20);
    a.x_keep = (uint32_t*)(g->xs + c * 24);
    a.x_list = (uint32_t*)(g->xs + c * 28);
    a.x_status = g->xs + c * 32;
    a.x_cap = c;
    // the extra names as "fragments" of D3 / D4
    x = a;
    x.n = c;
    x.svc_hash = a.x_hash;
    x.name_ptr = a.x_ptr;
    x.name_len = a.x_len;
    x.svc = a.x_svc;
    x.keep = a.x_keep;
    x.status = a.x_status;
    x.pub = a.x_list;
    x.pub_n = a.icnt + 3;
}

zk_status ingest_batch(zk_ingest_dev* g, const uint8_t* buf, const uint64_t* offsets, uint64_t n, uint32_t codec,
                       uint32_t flags, const zk_span_cols* out, uint64_t* n_out, uint64_t* n_rejected,
                       zk_ingest_items* items, const uint64_t* ends = nullptr) {
    if (!g || !n_out || !n_rejected) return ZK_ERR_INVALID_ARG;
    *n_out = *n_rejected = 0;
    if (items) items->kv_n = items->ann_n = 0;
    const bool want_kv = items && items->kv_service && items->kv_key && items->kv_cap;
    const bool want_ann = items && items->ann_service && items->ann_value && items->ann_cap;
    if (n == 0) return ZK_OK;
    if (items && n >= (1ull << 30)) return dfail(g, ZK_ERR_INVALID_ARG, "items: batch of 2^30 fragments or more");
    if (!buf || !offsets || !out || !out->trace_id || !out->span_id || !out->parent_id || !out->first_ts ||
        !out->last_ts || !out->service_id || !out->flags)
        return ZK_ERR_INVALID_ARG;
    if (codec != ZK_CODEC_THRIFT && codec != ZK_CODEC_SNAPPY_THRIFT) return dfail(g, ZK_ERR_INVALID_ARG, "unknown codec");
    if (n >= 0x7FFFFFFFull) return dfail(g, ZK_ERR_INVALID_ARG, "batch of 2^31 fragments or more");
    ING_HIP(g, hipSetDevice(g->device));
    // per-fragment arrays: 8-byte columns first, then 4-byte, then 1-byte
    const uint64_t n1 = n + 1;
    const uint64_t bytes = align256(8 * n1) * 8 + align256(4 * n1) * 9 + align256(n1);
    if (bytes > g->batch_cap) {
        hipFree(g->batch);
        g->batch = nullptr;
        ING_HIP(g, hipMalloc(&g->batch, bytes));
        g->batch_cap = bytes;
    }
    uint8_t* p = (uint8_t*)g->batch;
    auto take = [&](uint64_t b) {
        uint8_t* q = p;
        p += align256(b);
        return q;
    };
    IngArgs a{};
    a.buf = buf;
    a.offsets = offsets;
    a.ends = ends ? ends : offsets + 1;
    a.n = n;
    a.snappy = codec == ZK_CODEC_SNAPPY_THRIFT;
    // records are written straight into the caller's columns at their fragment index; when some
    // fragment is dropped they are copied here and compacted back (below)
    zk_span_cols tmp{};
    tmp.trace_id = (uint64_t*)take(8 * n1);
    tmp.span_id = (uint64_t*)take(8 * n1);
    tmp.parent_id = (uint64_t*)take(8 * n1);
    tmp.first_ts = (int64_t*)take(8 * n1);
    tmp.last_ts = (int64_t*)take(8 * n1);
    a.svc_hash = (uint64_t*)take(8 * n1);
    a.name_ptr = (uint64_t*)take(8 * n1);
    take(8 * n1);  // (spare)
    tmp.flags = (uint32_t*)take(4 * n1);
    tmp.service_id = (uint32_t*)take(4 * n1);
    a.name_len = (uint32_t*)take(4 * n1);
    a.tid = (uint64_t*)out->trace_id;
    a.sid = (uint64_t*)out->span_id;
    a.pid = (uint64_t*)out->parent_id;
    a.first = (int64_t*)out->first_ts;
    a.last = (int64_t*)out->last_ts;
    a.flags = (uint32_t*)out->flags;
    a.svc = (uint32_t*)out->service_id;
    a.keep = (uint32_t*)take(4 * n1);
    a.pos = (uint32_t*)take(4 * n1);
    a.pub = (uint32_t*)take(4 * n1);
    a.def = (uint32_t*)take(4 * n1);
    a.skip_kv = (uint32_t*)take(4 * n1);
    a.skip_an = (uint32_t*)take(4 * n1);
    a.status = take(n1);
    a.d_key = g->d_key;
    a.d_id = g->d_id;
    a.d_ptr = g->d_ptr;
    a.d_len = g->d_len;
    a.d_name16 = g->d_name16;
    a.d_mask = g->table - 1;
    a.max_services = g->max_services;
    a.unknown = g->arena;
    a.icnt = g->counts + 16;
    // fragments per wave of the LDS decoder: 1024 once a batch gives ~4096 waves (2 per wave slot of
    // 256 CUs x 8), else the power of two that does, at least 128 (~2 rounds of a wave)
    uint32_t lds_block = 128;
    while (lds_block < kLdsBlock && (uint64_t)lds_block * 4096 < n) lds_block <<= 1;
    IngArgs ax{};  // the extra names (items only)
    if (items) {
        a.items = 1;
        a.kv_cap = want_kv ? items->kv_cap : 0;
        a.an_cap = want_ann ? items->ann_cap : 0;
        // staging: the direct items (as many as the caller's buffers take) and the chunks (the
        // caller's capacity in chunks plus one partly filled chunk per LDS-decoder wave)
        const uint64_t waves = (n + lds_block - 1) / lds_block;  // the LDS decoder's workgroups (one wave each)
        const uint64_t ck_cap = (std::max(a.kv_cap, a.an_cap) + kItemChunk - 1) / kItemChunk + waves + 1;
        if (ck_cap > 0xFFFFFFF0ull) return dfail(g, ZK_ERR_INVALID_ARG, "items: item buffers too large");
        const uint64_t ck_items = ck_cap * kItemChunk;
        const uint64_t need_st = align256(a.kv_cap * 4) + align256(a.kv_cap * 8) + align256(a.an_cap * 4) +
                                 align256(a.an_cap * 8) + 2 * (align256(ck_items * 4) + align256(ck_items * 8) +
                                                               2 * align256(ck_cap * 4));
        if (need_st > g->istage_cap) {
            ING_HIP(g, hipStreamSynchronize(g->stream));  // (a previous batch's compaction may still read it)
            hipFree(g->istage);
            g->istage = nullptr;
            g->istage_cap = 0;
            ING_HIP(g, hipMalloc(&g->istage, need_st));
            g->istage_cap = need_st;
        }
        uint8_t* q = g->istage;
        auto takei = [&](uint64_t b) {
            uint8_t* r = q;
            q += align256(b);
            return r;
        };
        a.kv_svc = (uint32_t*)takei(a.kv_cap * 4);
        a.kv_key = (uint64_t*)takei(a.kv_cap * 8);
        a.an_svc = (uint32_t*)takei(a.an_cap * 4);
        a.an_val = (uint64_t*)takei(a.an_cap * 8);
        for (int k = 0; k < 2; ++k) {
            a.ck_svc[k] = (uint32_t*)takei(ck_items * 4);
            a.ck_key[k] = (uint64_t*)takei(ck_items * 8);
            a.ck_fill[k] = (uint32_t*)takei(ck_cap * 4);
            takei(ck_cap * 4);  // the fills' exclusive scan (ck_off below)
        }
        a.ck_cap = (uint32_t)ck_cap;
        if (!g->s_key) ING_HIP(g, grow_string_set(g, 1u << 16));
        while (g->s_count * 2 > g->s_cap) ING_HIP(g, grow_string_set(g, g->s_cap * 2));
        ING_HIP(g, size_new_strings(g, 0));
        if (!g->xs) ING_HIP(g, size_extra(g, 4096, 0));
        ING_HIP(g, hipMemsetAsync(a.icnt, 0, 13 * 8, g->stream));
    }
    const dim3 grid((unsigned)((n + kIngWG - 1) / kIngWG)), blk(kIngWG);
    const dim3 lgrid(std::min<unsigned>(grid.x, 2048u));  // the list kernels (grid-stride)
    hipStream_t s = g->stream;
    size_t need = 0;
    ING_HIP(g, hipcub::DeviceScan::ExclusiveSum(nullptr, need, a.keep, a.pos, (int)n1, s));
    if (need > g->cub_cap) {
        hipFree(g->cub);
        g->cub = nullptr;
        ING_HIP(g, hipMalloc(&g->cub, need));
        g->cub_cap = need;
    }
    if (a.snappy && !g->scratch) {
        const uint64_t cap = g->scratch_min ? g->scratch_min : std::max<uint64_t>(1ull << 26, 24 * n);
        ING_HIP(g, hipMalloc(&g->scratch, cap));
        g->scratch_cap = cap;
    }
    unsigned long long* used = g->counts + 10;
    ING_HIP(g, hipMemsetAsync(used, 0, 4 * 8, s));  // scratch taken, pub_n, def_n, claims
    a.pub_n = g->counts + 11;
    a.def_n = g->counts + 12;
    a.claims = g->counts + 13;
    a.scratch = g->scratch;
    a.scratch_cap = g->scratch_cap;
    a.scratch_used = used;
    if (items) bind_items(g, a, ax);  // (ax copies a: every field of a is set by now)
    // D1 + D2, D3
    a.lds_block = lds_block;
    const dim3 dgrid((unsigned)((n + a.lds_block - 1) / a.lds_block));
    if (items) {
        ING_HIP(g, launch_checked("k_ing_decode_lds", k_ing_decode_lds<true>, dgrid, dim3(kLdsWG), 0, s, a));
        ING_HIP(g, launch_checked("k_ing_decode", k_ing_decode<true>, lgrid, blk, 0, s, a, (uint32_t)kStDefer));
    } else {
        ING_HIP(g, launch_checked("k_ing_decode_lds", k_ing_decode_lds<false>, dgrid, dim3(kLdsWG), 0, s, a));
        ING_HIP(g, launch_checked("k_ing_decode", k_ing_decode<false>, lgrid, blk, 0, s, a, (uint32_t)kStDefer));
    }
    ING_HIP(g, launch_checked("k_ing_dict_insert", k_ing_dict_insert, lgrid, blk, 0, s, a));
    const dim3 xgrid(64);  // the extra-name list kernels (grid-stride; the list is short)
    if (items) ING_HIP(g, launch_checked("k_ing_dict_insert_x", k_ing_dict_insert_x, xgrid, blk, 0, s, ax));
    // D4 and the status counts, then one small read: in the steady state (no scratch overflow, no
    // new service names) this is the batch's only host round trip
    unsigned long long* const hc = g->h_counts;
    auto lookup_and_count = [&]() -> hipError_t {
        hipError_t e = launch_checked("k_ing_lookup", k_ing_lookup, lgrid, blk, 0, s, a);
        if (e == hipSuccess) e = hipMemsetAsync(g->counts, 0, 8 * 8, s);
        if (e == hipSuccess) e = hipMemsetAsync(g->counts + 8, 0xFF, 8, s);
        if (e == hipSuccess)
            e = launch_checked("k_ing_count", k_ing_count, grid, blk, 0, s, (const uint8_t*)a.status, n, g->counts,
                               (unsigned int*)(g->counts + 8));
        if (items) {
            if (e == hipSuccess) e = launch_checked("k_ing_lookup_x", k_ing_lookup_x, xgrid, blk, 0, s, ax);
            if (e == hipSuccess) e = hipMemsetAsync(a.icnt + 5, 0, 2 * 8, s);
            if (e == hipSuccess) e = launch_checked("k_ing_count_extra", k_ing_count_extra, xgrid, blk, 0, s, ax);
        }
        if (e == hipSuccess) e = hipMemcpyAsync(hc, g->counts, (items ? 29 : 14) * 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        return e;
    };
    ING_HIP(g, lookup_and_count());
    std::vector<uint8_t*> retired;  // old arenas and scratch stay valid until this batch's lookups are done
    unsigned long long* const ic = hc + 16;  // the host copy of a.icnt
    auto items_short = [&]() { return items && (ic[4] > 0 || ic[3] > g->x_cap); };
    if (hc[10] > g->scratch_cap || hc[13] > 0 || items_short()) {
        while (hc[10] > g->scratch_cap || items_short()) {
            // the scratch ran out (kStNoScratch fragments): a larger one, and those fragments again
            if (hc[10] > g->scratch_cap) {
                uint64_t cap = 2 * g->scratch_cap;
                if (cap < hc[10]) cap = hc[10];
                retired.push_back(g->scratch);
                g->scratch = nullptr;
                g->scratch_cap = 0;
                ING_HIP(g, hipMalloc(&g->scratch, cap));
                g->scratch_cap = cap;
                ING_HIP(g, hipMemsetAsync(used, 0, 8, s));
                a.scratch = g->scratch;
                a.scratch_cap = cap;
            }
            if (items_short()) {  // the string set or the extra list filled up: larger ones
                if (ic[3] > g->x_cap) {
                    const uint64_t old = g->x_cap;
                    ING_HIP(g, size_extra(g, std::max<uint64_t>(2 * old, 2 * ic[3]), old));
                    ING_HIP(g, hipMemcpyAsync(a.icnt + 3, &old, 8, hipMemcpyHostToDevice, s));
                    ING_HIP(g, hipStreamSynchronize(s));
                }
                if (ic[4] > 0) {
                    ING_HIP(g, grow_string_set(g, g->s_cap * 2));
                    ING_HIP(g, size_new_strings(g, std::min<uint64_t>(ic[2], g->ns_cap)));
                }
                ING_HIP(g, hipMemsetAsync(a.icnt + 4, 0, 8, s));
                ING_HIP(g, hipStreamSynchronize(s));
                bind_items(g, a, ax);
            }
            ING_HIP(g, launch_checked("k_ing_decode", items ? k_ing_decode<true> : k_ing_decode<false>, lgrid, blk, 0, s,
                                      a, (uint32_t)kStNoScratch));
            ING_HIP(g, launch_checked("k_ing_dict_insert", k_ing_dict_insert, lgrid, blk, 0, s, a));
            if (items) ING_HIP(g, launch_checked("k_ing_dict_insert_x", k_ing_dict_insert_x, xgrid, blk, 0, s, ax));
            ING_HIP(g, hipMemcpyAsync(hc + 10, used, (items ? 19 : 1) * 8, hipMemcpyDeviceToHost, s));
            ING_HIP(g, hipStreamSynchronize(s));
        }
        // ids for new slots, in slot order; their names into the device arena
        std::vector<uint64_t> key(g->table), ptr(g->table);
        std::vector<uint32_t> len(g->table);
        ING_HIP(g, hipMemcpyAsync(key.data(), g->d_key, key.size() * 8, hipMemcpyDeviceToHost, s));
        ING_HIP(g, hipMemcpyAsync(ptr.data(), g->d_ptr, ptr.size() * 8, hipMemcpyDeviceToHost, s));
        ING_HIP(g, hipMemcpyAsync(len.data(), g->d_len, len.size() * 4, hipMemcpyDeviceToHost, s));
        ING_HIP(g, hipStreamSynchronize(s));
        // the new slots in slot order, their names gathered into the arena by one kernel and read
        // back in one copy
        std::vector<uint32_t> fresh;
        uint64_t total = 0;
        for (uint32_t q = 0; q < g->table; ++q)
            if (key[q] != kEmpty && g->slot_id[q] == kNoId) {
                fresh.push_back(q);
                total += len[q];
            }
        const bool changed = !fresh.empty();
        if (changed) {
            if (g->arena_used + total > g->arena_cap) {
                uint64_t cap = g->arena_cap;
                while (cap < g->arena_used + total) cap *= 2;
                uint8_t* na = nullptr;
                ING_HIP(g, hipMalloc(&na, cap));
                ING_HIP(g, hipMemcpyAsync(na, g->arena, g->arena_used, hipMemcpyDeviceToDevice, s));
                // repoint the named slots at the new arena
                for (uint32_t r = 0; r < g->table; ++r)
                    if (g->slot_id[r] != kNoId)
                        ptr[r] = (uint64_t)(uintptr_t)na + (ptr[r] - (uint64_t)(uintptr_t)g->arena);
                retired.push_back(g->arena);
                g->arena = na;
                g->arena_cap = cap;
                a.unknown = na;
            }
            const uint32_t m = (uint32_t)fresh.size();
            std::vector<uint64_t> gsrc(m), goff(m);
            std::vector<uint32_t> glen(m);
            uint64_t at = g->arena_used;
            for (uint32_t k = 0; k < m; ++k) {
                gsrc[k] = ptr[fresh[k]];
                goff[k] = at;
                glen[k] = len[fresh[k]];
                at += glen[k];
            }
            uint8_t* gt = nullptr;  // the gather's table: sources, arena offsets, lengths
            ING_HIP(g, hipMalloc(&gt, (uint64_t)m * 20));
            retired.push_back(gt);
            ING_HIP(g, hipMemcpyAsync(gt, gsrc.data(), (uint64_t)m * 8, hipMemcpyHostToDevice, s));
            ING_HIP(g, hipMemcpyAsync(gt + (uint64_t)m * 8, goff.data(), (uint64_t)m * 8, hipMemcpyHostToDevice, s));
            ING_HIP(g, hipMemcpyAsync(gt + (uint64_t)m * 16, glen.data(), (uint64_t)m * 4, hipMemcpyHostToDevice, s));
            ING_HIP(g, launch_checked("k_ing_gather_names", k_ing_gather_names, dim3((m + 255) / 256), dim3(256), 0, s,
                                      (const uint64_t*)gt, (const uint64_t*)(gt + (uint64_t)m * 8),
                                      (const uint32_t*)(gt + (uint64_t)m * 16), m, g->arena));
            std::string bytes(total, '\0');
            if (total)
                ING_HIP(g, hipMemcpyAsync(&bytes[0], g->arena + g->arena_used, total, hipMemcpyDeviceToHost, s));
            ING_HIP(g, hipStreamSynchronize(s));
            for (uint32_t k = 0; k < m; ++k) {
                const uint32_t q = fresh[k];
                std::string nm = bytes.substr(goff[k] - g->arena_used, glen[k]);
                ptr[q] = (uint64_t)(uintptr_t)(g->arena + goff[k]);
                g->slot_id[q] = (uint32_t)g->names.size();
                memcpy(&g->name16[(size_t)q * 16], nm.data(), std::min<size_t>(16, nm.size()));
                g->names.push_back(std::move(nm));
            }
            g->arena_used = at;
        }
        if (changed) {
            ING_HIP(g, hipMemcpyAsync(g->d_id, g->slot_id.data(), g->slot_id.size() * 4, hipMemcpyHostToDevice, s));
            ING_HIP(g, hipMemcpyAsync(g->d_ptr, ptr.data(), ptr.size() * 8, hipMemcpyHostToDevice, s));
            ING_HIP(g, hipMemcpyAsync(g->d_name16, g->name16.data(), g->name16.size(), hipMemcpyHostToDevice, s));
        }
        ING_HIP(g, lookup_and_count());  // D4 again, now that every claimed slot has its id
    }
    unsigned long long c[9];
    memcpy(c, hc, sizeof(c));
    unsigned long long icf[13] = {0};
    if (items) memcpy(icf, ic, sizeof(icf));
    if (items && icf[2]) {
        // the strings captured in this batch -> the host map (before any error return: their hashes
        // are in the device set from now on)
        const uint64_t m = std::min<uint64_t>(icf[2], g->ns_cap);
        std::vector<uint64_t> hh(m), pp(m), off(m);
        std::vector<uint32_t> ll(m);
        ING_HIP(g, hipMemcpyAsync(hh.data(), a.ns_hash, m * 8, hipMemcpyDeviceToHost, s));
        ING_HIP(g, hipMemcpyAsync(pp.data(), a.ns_ptr, m * 8, hipMemcpyDeviceToHost, s));
        ING_HIP(g, hipMemcpyAsync(ll.data(), a.ns_len, m * 4, hipMemcpyDeviceToHost, s));
        ING_HIP(g, hipStreamSynchronize(s));
        uint64_t total = 0;
        for (uint64_t k = 0; k < m; ++k) {
            off[k] = total;
            total += ll[k];
        }
        std::string bytes(total, '\0');
        if (total) {
            uint8_t* gt = nullptr;  // destination offsets, then the gathered bytes
            ING_HIP(g, hipMalloc(&gt, m * 8 + total));
            retired.push_back(gt);
            ING_HIP(g, hipMemcpyAsync(gt, off.data(), m * 8, hipMemcpyHostToDevice, s));
            ING_HIP(g, launch_checked("k_ing_gather_names", k_ing_gather_names, dim3((unsigned)((m + 255) / 256)), dim3(256),
                                      0, s, (const uint64_t*)a.ns_ptr, (const uint64_t*)gt, (const uint32_t*)a.ns_len,
                                      (uint32_t)m, gt + m * 8));
            ING_HIP(g, hipMemcpyAsync(&bytes[0], gt + m * 8, total, hipMemcpyDeviceToHost, s));
            ING_HIP(g, hipStreamSynchronize(s));
        }
        for (uint64_t k = 0; k < m; ++k) g->strings.emplace(hh[k], bytes.substr(off[k], ll[k]));
        g->s_count += m;
    }
    for (uint8_t* r : retired) hipFree(r);
    uint64_t dropped = 0;  // every fragment whose status is not ok is not a record
    for (int q = 0; q < 8; ++q) dropped += c[q];
    const uint64_t kept = n - dropped;
    const unsigned first_bad = (unsigned)(c[8] & 0xFFFFFFFFu);
    if (c[kStCollision])
        return dfail(g, ZK_ERR_INVALID_SPAN, "two service names share a 64-bit hash (fragment " +
                                                  std::to_string(first_bad) + ")");
    if (icf[5]) return dfail(g, ZK_ERR_INVALID_SPAN, "two service names (an item's host) share a 64-bit hash");
    if (c[kStRange] || icf[6])
        return dfail(g, ZK_ERR_SERVICE_RANGE, "more distinct service names than max_services");
    const bool strict = (flags & ZK_INGEST_STRICT) != 0;
    const uint64_t bad = c[kStInvalid] + c[kStUndecodable];
    if (strict && bad)
        return dfail(g, ZK_ERR_INVALID_SPAN, "span " + std::to_string(first_bad) + ": " +
                                                 (c[kStUndecodable] ? "undecodable or invalid span" : "invalid span"));
    uint64_t nkv = 0, nan = 0, tot[2] = {0, 0};
    if (items) {
        // the chunks and the direct items into the caller's buffers (k_ing_item_compact), then the item
        // services' references -> ids (k_ing_item_fixup, on the caller's buffers)
        uint32_t* out_s[2] = {items->kv_service, items->ann_service};
        uint64_t* out_k[2] = {items->kv_key, items->ann_value};
        const uint64_t cap[2] = {a.kv_cap, a.an_cap};
        for (int k = 0; k < 2; ++k) {
            if (!cap[k]) continue;
            const uint32_t nch = (uint32_t)std::min<uint64_t>(icf[11 + k], a.ck_cap);
            uint32_t* off = a.ck_fill[k] + align256((uint64_t)a.ck_cap * 4) / 4;
            if (nch) {
                size_t nb = 0;
                ING_HIP(g, hipcub::DeviceScan::ExclusiveSum(nullptr, nb, a.ck_fill[k], off, (int)nch, s));
                if (nb > g->cub_cap) {
                    ING_HIP(g, hipStreamSynchronize(s));
                    hipFree(g->cub);
                    g->cub = nullptr;
                    ING_HIP(g, hipMalloc(&g->cub, nb));
                    g->cub_cap = nb;
                }
                ING_HIP(g, hipcub::DeviceScan::ExclusiveSum(g->cub, nb, a.ck_fill[k], off, (int)nch, s));
            }
            const uint64_t nd = std::min<uint64_t>(icf[k], cap[k]);
            const uint64_t work = (uint64_t)nch * kItemChunk + nd;
            ING_HIP(g, launch_checked("k_ing_item_compact", k_ing_item_compact,
                                      dim3((unsigned)std::max<uint64_t>(1, std::min<uint64_t>((work + kIngWG - 1) / kIngWG, 8192))),
                                      blk, 0, s, a, (uint32_t)k, nch, (const uint32_t*)off, nd, out_s[k], out_k[k], cap[k]));
        }
        ING_HIP(g, hipMemcpyAsync(hc + 25, a.icnt + 9, 2 * 8, hipMemcpyDeviceToHost, s));
        ING_HIP(g, hipStreamSynchronize(s));
        for (int k = 0; k < 2; ++k) tot[k] = cap[k] ? hc[25 + k] + icf[k] + icf[7 + k] : 0;
        nkv = std::min<uint64_t>(tot[0], cap[0]);
        nan = std::min<uint64_t>(tot[1], cap[1]);
        a.kv_svc = items->kv_service;
        a.an_svc = items->ann_service;
    }
    if (nkv + nan) {  // item services (references to a fragment's record or an extra name) -> ids
        ING_HIP(g, launch_checked("k_ing_item_fixup", k_ing_item_fixup,
                                  dim3((unsigned)std::min<uint64_t>((nkv + nan + kIngWG - 1) / kIngWG, 4096)), blk, 0, s,
                                  a, nkv, nan));
        if (!dropped) ING_HIP(g, hipStreamSynchronize(s));
    }
    if (dropped) {
        // D5: the records sit at their fragment index in the caller's columns; copy them aside and
        // compact them back in input order
        ING_HIP(g, hipMemsetAsync(a.keep + n, 0, 4, s));
        ING_HIP(g, hipcub::DeviceScan::ExclusiveSum(g->cub, need, a.keep, a.pos, (int)n1, s));
        ING_HIP(g, hipMemcpyAsync((void*)tmp.trace_id, out->trace_id, 8 * n, hipMemcpyDeviceToDevice, s));
        ING_HIP(g, hipMemcpyAsync((void*)tmp.span_id, out->span_id, 8 * n, hipMemcpyDeviceToDevice, s));
        ING_HIP(g, hipMemcpyAsync((void*)tmp.parent_id, out->parent_id, 8 * n, hipMemcpyDeviceToDevice, s));
        ING_HIP(g, hipMemcpyAsync((void*)tmp.first_ts, out->first_ts, 8 * n, hipMemcpyDeviceToDevice, s));
        ING_HIP(g, hipMemcpyAsync((void*)tmp.last_ts, out->last_ts, 8 * n, hipMemcpyDeviceToDevice, s));
        ING_HIP(g, hipMemcpyAsync((void*)tmp.service_id, out->service_id, 4 * n, hipMemcpyDeviceToDevice, s));
        ING_HIP(g, hipMemcpyAsync((void*)tmp.flags, out->flags, 4 * n, hipMemcpyDeviceToDevice, s));
        a.tid = (uint64_t*)tmp.trace_id;
        a.sid = (uint64_t*)tmp.span_id;
        a.pid = (uint64_t*)tmp.parent_id;
        a.first = (int64_t*)tmp.first_ts;
        a.last = (int64_t*)tmp.last_ts;
        a.flags = (uint32_t*)tmp.flags;
        a.svc = (uint32_t*)tmp.service_id;
        ING_HIP(g, launch_checked("k_ing_compact", k_ing_compact, grid, blk, 0, s, a, *out));
        ING_HIP(g, hipStreamSynchronize(s));
    }
    *n_out = kept;
    *n_rejected = bad;
    if (items) {
        items->kv_n = nkv;
        items->ann_n = nan;
        if ((want_kv && tot[0] > a.kv_cap) || (want_ann && tot[1] > a.an_cap))
            return dfail(g, ZK_ERR_CAPACITY, "item buffers too small: " + std::to_string(tot[0]) + " key-value and " +
                                                 std::to_string(tot[1]) + " annotation items");
    }
    return ZK_OK;
}

// zk_ingest_dev_spans_multi: the batches' extents joined into starts / ends (one small kernel), then
// one decode over all of them
zk_status ingest_multi(zk_ingest_dev* g, uint32_t nb, const uint8_t* const* bufs, const uint64_t* const* offsets,
                       const uint64_t* ns, uint32_t codec, uint32_t flags, const zk_span_cols* out, uint64_t* n_out,
                       uint64_t* n_rejected, zk_ingest_items* items) {
    if (!g || !n_out || !n_rejected) return ZK_ERR_INVALID_ARG;
    *n_out = *n_rejected = 0;
    if (items) items->kv_n = items->ann_n = 0;
    if (nb && (!bufs || !offsets || !ns)) return dfail(g, ZK_ERR_INVALID_ARG, "null batch arrays");
    uint64_t n = 0;
    uintptr_t base = UINTPTR_MAX;
    uint32_t only = nb;  // the one non-empty batch, if there is exactly one
    for (uint32_t b = 0; b < nb; ++b) {
        if (!ns[b]) continue;
        if (!bufs[b] || !offsets[b]) return dfail(g, ZK_ERR_INVALID_ARG, "batch " + std::to_string(b) + ": null buffer");
        if (ns[b] >= 0x7FFFFFFFull - n) return dfail(g, ZK_ERR_INVALID_ARG, "batches of 2^31 fragments or more");
        n += ns[b];
        base = std::min(base, (uintptr_t)bufs[b]);
        only = only == nb ? b : nb + 1;
    }
    if (n == 0) return ZK_OK;
    if (only < nb)  // one batch: its own extents
        return ingest_batch(g, bufs[only], offsets[only], ns[only], codec, flags, out, n_out, n_rejected, items);
    ING_HIP(g, hipSetDevice(g->device));
    const uint64_t tab_bytes = align256((uint64_t)nb * sizeof(IngMultiBatch));
    const uint64_t need = tab_bytes + 2 * align256(8 * n);
    if (need > g->multi_cap) {
        ING_HIP(g, hipStreamSynchronize(g->stream));  // (a previous call's decode may still read it)
        hipFree(g->multi);
        g->multi = nullptr;
        g->multi_cap = 0;
        ING_HIP(g, hipMalloc(&g->multi, need));
        g->multi_cap = need;
    }
    std::vector<IngMultiBatch> tab(nb);
    uint64_t first = 0;
    for (uint32_t b = 0; b < nb; ++b) {
        tab[b].rel = ns[b] ? (uint64_t)((uintptr_t)bufs[b] - base) : 0;
        tab[b].offsets = offsets[b];
        tab[b].first = first;
        first += ns[b];
    }
    IngMultiBatch* dtab = (IngMultiBatch*)g->multi;
    uint64_t* starts = (uint64_t*)(g->multi + tab_bytes);
    uint64_t* ends = (uint64_t*)(g->multi + tab_bytes + align256(8 * n));
    // the table from pageable memory; the decode below synchronises before this call returns
    ING_HIP(g, hipMemcpyAsync(dtab, tab.data(), (uint64_t)nb * sizeof(IngMultiBatch), hipMemcpyHostToDevice, g->stream));
    ING_HIP(g, launch_checked("k_ing_multi_bounds", k_ing_multi_bounds, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                              g->stream, (const IngMultiBatch*)dtab, nb, n, starts, ends));
    const zk_status st = ingest_batch(g, (const uint8_t*)base, starts, n, codec, flags, out, n_out, n_rejected, items, ends);
    if (st != ZK_OK) hipStreamSynchronize(g->stream);  // (an early error return: the table copy is done)
    return st;
}

}  // namespace

extern "C" {

zk_status zk_ingest_dev_spans_multi(zk_ingest_dev* g, uint32_t nb, const uint8_t* const* bufs,
                                    const uint64_t* const* offsets, const uint64_t* ns, uint32_t codec, uint32_t flags,
                                    const zk_span_cols* out, uint64_t* n_out, uint64_t* n_rejected,
                                    zk_ingest_items* items) {
    ZK_GUARD_BEGIN
    return ingest_multi(g, nb, bufs, offsets, ns, codec, flags, out, n_out, n_rejected, items);
    ZK_GUARD_END
}

zk_status zk_ingest_dev_spans(zk_ingest_dev* g, const uint8_t* buf, const uint64_t* offsets, uint64_t n,
                              uint32_t codec, uint32_t flags, const zk_span_cols* out, uint64_t* n_out,
                              uint64_t* n_rejected) {
    ZK_GUARD_BEGIN
    return ingest_batch(g, buf, offsets, n, codec, flags, out, n_out, n_rejected, nullptr);
    ZK_GUARD_END
}

zk_status zk_ingest_dev_spans_items(zk_ingest_dev* g, const uint8_t* buf, const uint64_t* offsets, uint64_t n,
                                    uint32_t codec, uint32_t flags, const zk_span_cols* out, uint64_t* n_out,
                                    uint64_t* n_rejected, zk_ingest_items* items) {
    ZK_GUARD_BEGIN
    if (!items) return ZK_ERR_INVALID_ARG;
    return ingest_batch(g, buf, offsets, n, codec, flags, out, n_out, n_rejected, items);
    ZK_GUARD_END
}

zk_status zk_ingest_dev_string(const zk_ingest_dev* g, uint64_t hash, char* buf, uint64_t cap, uint64_t* len) {
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

zk_status zk_ingest_dev_num_services(const zk_ingest_dev* g, uint32_t* n) {
    ZK_GUARD_BEGIN
    if (!g || !n) return ZK_ERR_INVALID_ARG;
    *n = (uint32_t)g->names.size();
    return ZK_OK;
    ZK_GUARD_END
}

zk_status zk_ingest_dev_service_name(const zk_ingest_dev* g, uint32_t id, char* buf, uint64_t cap, uint64_t* len) {
    ZK_GUARD_BEGIN
    if (!g || !len) return ZK_ERR_INVALID_ARG;
    if (id >= g->names.size()) return ZK_ERR_SERVICE_RANGE;
    const std::string& s = g->names[id];
    *len = s.size();
    if (!buf) return ZK_OK;
    if (cap < s.size()) return ZK_ERR_CAPACITY;
    memcpy(buf, s.data(), s.size());
    return ZK_OK;
    ZK_GUARD_END
}

}  // extern "C"
