// fuzz_host.cpp — ASan/UBSan driver for the host-side byte parsers and the store (CPU only).
//
// Built by tools/sanitize/Makefile from the product sources zk_ingest.cpp and zk_store.cpp plus the
// oracle's zk_oracle.c, with -fsanitize=address,undefined and no recovery: any out-of-bounds access,
// use-after-free, leak or undefined behaviour aborts the run. Input: a corpus file of length-prefixed
// stored fragments (u32 little-endian length, then the bytes), written by tests/test_sanitize.py from
// the thrift encoder. Every fragment is decoded as is, Snappy-compressed by the corpus writer's
// choice, and under deterministic mutations (bit flips, truncation, splices, hostile Snappy headers),
// through both codecs, strict and lenient, with the indexer items on.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "zkingest.h"
#include "zkstore.h"

extern "C" int zko_aggregate(const uint64_t* tid, const uint64_t* sid, const uint64_t* pid, const int64_t* first,
                             const int64_t* last, const uint32_t* svc, const uint32_t* flags, uint64_t n, uint32_t S,
                             int threads, uint64_t* cells, uint64_t* stats);

namespace {

uint64_t g_rng = 0x9E3779B97F4A7C15ull;
uint64_t rnd() {
    uint64_t z = (g_rng += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Batch {
    std::vector<uint8_t> buf;
    std::vector<uint64_t> off{0};
    void add(const std::vector<uint8_t>& b) {
        buf.insert(buf.end(), b.begin(), b.end());
        off.push_back(buf.size());
    }
};

uint64_t decode(zk_ingest* g, const Batch& b, uint32_t codec, uint32_t flags) {
    const uint64_t n = b.off.size() - 1;
    std::vector<uint64_t> tid(n), sid(n), pid(n);
    std::vector<int64_t> f(n), l(n);
    std::vector<uint32_t> svc(n), fl(n);
    zk_span_cols out{tid.data(), sid.data(), pid.data(), f.data(), l.data(), svc.data(), fl.data(), n};
    const uint64_t cap = 4 * n + 4;
    std::vector<uint32_t> ks(cap), as(cap);
    std::vector<uint64_t> kk(cap), av(cap);
    zk_ingest_items it{ks.data(), kk.data(), cap, 0, as.data(), av.data(), cap, 0};
    uint64_t nout = 0, nrej = 0;
    const uint8_t* p = b.buf.empty() ? (const uint8_t*)"" : b.buf.data();
    zk_ingest_spans(g, p, b.off.data(), n, codec, flags, &out, &nout, &nrej, &it);
    if (nout > n) abort();
    return nout;
}

std::vector<uint8_t> mutate(const std::vector<uint8_t>& in) {
    std::vector<uint8_t> b = in;
    switch (rnd() % 5) {
        case 0:
            for (int k = 0, m = 1 + (int)(rnd() % 6); k < m && !b.empty(); ++k) b[rnd() % b.size()] ^= (uint8_t)rnd();
            break;
        case 1:
            if (!b.empty()) b.resize(rnd() % b.size());
            break;
        case 2: {  // splice a random window over another position
            if (b.size() > 4) {
                const size_t a = rnd() % b.size(), c = rnd() % b.size(), len = rnd() % (b.size() - (a > c ? a : c));
                memmove(&b[c], &b[a], len);
            }
            break;
        }
        case 3: {  // hostile Snappy header: a varint announcing up to 4 GiB
            uint64_t v = rnd() & 0xFFFFFFFFull;
            std::vector<uint8_t> h;
            while (v >= 0x80) {
                h.push_back((uint8_t)(v | 0x80));
                v >>= 7;
            }
            h.push_back((uint8_t)v);
            b.insert(b.begin(), h.begin(), h.end());
            break;
        }
        default:  // random bytes
            b.resize(rnd() % 64);
            for (auto& x : b) x = (uint8_t)rnd();
    }
    return b;
}

void fuzz_store() {
    for (uint32_t mode = 0; mode < 3; ++mode) {
        zk_store* s = nullptr;
        if (zk_store_create(mode, &s) != ZK_OK) abort();
        for (int r = 0; r < 200; ++r) {
            std::vector<zk_dep_link> links(rnd() % 20);
            for (auto& l : links)
                l = zk_dep_link{(uint32_t)(rnd() % 7), (uint32_t)(rnd() % 7),
                                zk_moments{(int64_t)(rnd() % 100 + 1), (double)(rnd() % 1000), 1.0, 2.0, 3.0}};
            const int64_t t = (int64_t)(rnd() % 2000000000000ull) - 1000000000;
            zk_store_put_dependencies(s, t, t + (int64_t)(rnd() % 1000000), links.data(), links.size());
            int64_t a = (int64_t)(rnd() % 3000000000000ull) - 1000000000, e = a + (int64_t)(rnd() % 4000000000ull);
            uint64_t n = 0;
            int64_t os, oe;
            zk_store_get_dependencies(s, (rnd() & 1) ? &a : nullptr, (rnd() & 1) ? &e : nullptr, 1500000000000, nullptr, 0,
                                      &n, &os, &oe);
            std::vector<zk_dep_link> out(n + 1);
            zk_store_get_dependencies(s, &a, &e, 1500000000000, out.data(), out.size(), &n, &os, &oe);
            std::vector<uint64_t> ids(rnd() % 8);
            for (auto& x : ids) x = rnd();
            zk_store_put_top(s, (uint32_t)(rnd() % 3), (uint32_t)(rnd() % 5), ids.data(), ids.size());
            uint64_t k = 0, got[16];
            zk_store_get_top(s, (uint32_t)(rnd() % 2), (uint32_t)(rnd() % 5), got, 16, &k);
            uint64_t cnt;
            int64_t wm;
            zk_store_count(s, &cnt);
            zk_store_watermark(s, &wm);
        }
        zk_store_destroy(s);
    }
}

void fuzz_oracle() {
    const uint64_t n = 20000;
    std::vector<uint64_t> tid(n), sid(n), pid(n);
    std::vector<int64_t> f(n), l(n);
    std::vector<uint32_t> svc(n), fl(n);
    for (uint64_t i = 0; i < n; ++i) {
        tid[i] = rnd() % 500;
        sid[i] = rnd() % 3000;
        pid[i] = rnd() % 3000;
        f[i] = (int64_t)(rnd() % 1000000);
        l[i] = f[i] + (int64_t)(rnd() % (1ull << 42));  // some beyond the 2^40 us range
        svc[i] = (uint32_t)(rnd() % 40);                 // some beyond S = 31
        fl[i] = (uint32_t)rnd() & 0xFF0Fu;
    }
    const uint32_t S = 31;
    std::vector<uint64_t> cells((size_t)S * S * 17), stats(16);
    if (zko_aggregate(tid.data(), sid.data(), pid.data(), f.data(), l.data(), svc.data(), fl.data(), n, S, 4,
                      cells.data(), stats.data()) != 0)
        abort();
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s corpus iterations\n", argv[0]);
        return 2;
    }
    FILE* fp = fopen(argv[1], "rb");
    if (!fp) return 2;
    std::vector<std::vector<uint8_t>> corpus;
    for (;;) {
        uint32_t len;
        if (fread(&len, 4, 1, fp) != 1) break;
        std::vector<uint8_t> b(len);
        if (len && fread(b.data(), 1, len, fp) != len) return 2;
        corpus.push_back(std::move(b));
    }
    fclose(fp);
    if (corpus.empty()) return 2;
    const long iters = atol(argv[2]);
    zk_ingest* g = nullptr;
    if (zk_ingest_create(&g) != ZK_OK) return 2;
    uint64_t decoded = 0;
    // the corpus as is (every entry must decode in lenient mode with its own codec)
    for (uint32_t codec = 0; codec < 2; ++codec) {
        Batch b;
        for (const auto& c : corpus) b.add(c);
        decoded += decode(g, b, codec, 0);
        decoded += decode(g, b, codec, ZK_INGEST_STRICT);
    }
    // large batches: the decoder's thread pool (contiguous ranges, one ordered commit), clean and
    // with mutated fragments spread over the ranges, against the one-thread decode
    for (int rep = 0; rep < 3; ++rep) {
        Batch b;
        while (b.off.size() < 40001) {
            const auto& c = corpus[rnd() % corpus.size()];
            b.add(rep && rnd() % 8 == 0 ? mutate(c) : c);
        }
        for (uint32_t codec = 0; codec < 2; ++codec) {
            decoded += decode(g, b, codec, 0);
            decoded += decode(g, b, codec, ZK_INGEST_ONE_THREAD);
            decoded += decode(g, b, codec, ZK_INGEST_STRICT);
        }
    }
    for (long it = 0; it < iters; ++it) {
        Batch b;
        const int m = 1 + (int)(rnd() % 16);
        for (int k = 0; k < m; ++k) b.add(mutate(corpus[rnd() % corpus.size()]));
        const uint32_t codec = (uint32_t)(rnd() & 1);
        decoded += decode(g, b, codec, (uint32_t)(rnd() & 1));
        const auto& one = b.buf;
        uint64_t len = 0;
        if (!one.empty() && zk_snappy_uncompress(one.data(), one.size(), nullptr, 0, &len) == ZK_OK) {
            std::vector<uint8_t> out(len + 1);
            zk_snappy_uncompress(one.data(), one.size(), out.data(), out.size(), &len);
        }
        int64_t s0, e0;
        uint64_t nl = 0;
        std::vector<zk_dep_link> links(64);
        if (!one.empty()) zk_dependencies_decode(g, one.data(), one.size(), &s0, &e0, links.data(), links.size(), &nl);
    }
    zk_ingest_destroy(g);
    fuzz_store();
    fuzz_oracle();
    printf("sanitized run ok: %zu corpus fragments, %ld mutated batches, %llu records decoded\n", corpus.size(), iters,
           (unsigned long long)decoded);
    return 0;
}
