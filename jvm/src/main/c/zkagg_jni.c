/*
 * zkagg_jni.c — the native side of com.twitter.zipkin.gpu.ZkNative: each JNI entry forwards to the
 * C ABI of libzkagg (include/zkagg.h, zkstore.h, zkingest.h) without adding semantics.
 *
 * NOT COMPILED IN THIS REPOSITORY: the build image has no jni.h (no JDK). A
 * maintainer builds it with
 *   cc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *      jvm/src/main/c/zkagg_jni.c -Lzipkin_amd -lzkagg -o libzkagg_jni.so
 * tests/test_abi.py checks that every zk_* function called here is declared in include/*.h.
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "zkagg.h"
#include "zkcomm.h"
#include "zkingest.h"
#include "zksketch.h"
#include "zkstore.h"

#define FN(name) Java_com_twitter_zipkin_gpu_ZkNative_00024_##name
#define CTX(h) ((zk_ctx*)(intptr_t)(h))
#define ING(h) ((zk_ingest*)(intptr_t)(h))
#define STORE(h) ((zk_store*)(intptr_t)(h))
#define COMM(h) ((zk_comm*)(intptr_t)(h))
#define RL(h) ((zk_rl*)(intptr_t)(h))
#define BUF(b) ((*env)->GetDirectBufferAddress(env, (b)))

/* ---- dependency job ---------------------------------------------------------------------------- */
JNIEXPORT jlong JNICALL FN(ctxCreate)(JNIEnv* env, jobject self, jint S, jint dev, jboolean strict, jint maxTrace) {
    zk_config c;
    zk_ctx* h = NULL;
    memset(&c, 0, sizeof(c));
    c.num_services = (uint32_t)S;
    c.device = dev;
    c.strict = strict ? 1u : 0u;
    c.max_trace_records = (uint32_t)maxTrace;
    return zk_ctx_create(&c, &h) == ZK_OK ? (jlong)(intptr_t)h : 0;
}

JNIEXPORT jint JNICALL FN(ctxDestroy)(JNIEnv* env, jobject self, jlong h) { return zk_ctx_destroy(CTX(h)); }

JNIEXPORT jstring JNICALL FN(lastError)(JNIEnv* env, jobject self, jlong h) {
    return (*env)->NewStringUTF(env, zk_last_error(CTX(h)));
}

JNIEXPORT jint JNICALL FN(reset)(JNIEnv* env, jobject self, jlong h) { return zk_deps_reset(CTX(h)); }

JNIEXPORT jint JNICALL FN(accumulate)(JNIEnv* env, jobject self, jlong h, jobject tid, jobject sid, jobject pid,
                                     jobject fts, jobject lts, jobject svc, jobject flg, jlong n, jint batchFlags) {
    zk_span_cols cols = {BUF(tid), BUF(sid), BUF(pid), BUF(fts), BUF(lts), BUF(svc), BUF(flg), (uint64_t)n};
    return zk_deps_accumulate(CTX(h), &cols, (uint32_t)batchFlags);
}

JNIEXPORT jint JNICALL FN(finalizeTable)(JNIEnv* env, jobject self, jlong h, jlongArray m0, jdoubleArray m1,
                                        jdoubleArray m2, jdoubleArray m3, jdoubleArray m4, jbyteArray present) {
    zk_link_table t;
    memset(&t, 0, sizeof(t));
    t.m0 = (uint64_t*)(*env)->GetLongArrayElements(env, m0, NULL);
    t.m1 = (*env)->GetDoubleArrayElements(env, m1, NULL);
    t.m2 = (*env)->GetDoubleArrayElements(env, m2, NULL);
    t.m3 = (*env)->GetDoubleArrayElements(env, m3, NULL);
    t.m4 = (*env)->GetDoubleArrayElements(env, m4, NULL);
    t.present = (uint8_t*)(*env)->GetByteArrayElements(env, present, NULL);
    const jint st = zk_deps_finalize(CTX(h), &t);
    (*env)->ReleaseLongArrayElements(env, m0, (jlong*)t.m0, 0);
    (*env)->ReleaseDoubleArrayElements(env, m1, t.m1, 0);
    (*env)->ReleaseDoubleArrayElements(env, m2, t.m2, 0);
    (*env)->ReleaseDoubleArrayElements(env, m3, t.m3, 0);
    (*env)->ReleaseDoubleArrayElements(env, m4, t.m4, 0);
    (*env)->ReleaseByteArrayElements(env, present, (jbyte*)t.present, 0);
    return st;
}

JNIEXPORT jint JNICALL FN(stats)(JNIEnv* env, jobject self, jlong h, jlongArray out) {
    zk_stats s;
    const jint st = zk_ctx_stats(CTX(h), &s);
    if (st == ZK_OK) {
        const jsize n = (*env)->GetArrayLength(env, out);
        const jsize have = (jsize)(sizeof(s) / sizeof(uint64_t));
        (*env)->SetLongArrayRegion(env, out, 0, n < have ? n : have, (const jlong*)&s);
    }
    return st;
}

/* the exchange form for a host that runs its own collective: out[0] = device pointer, out[1] = bytes */
JNIEXPORT jint JNICALL FN(depsPartial)(JNIEnv* env, jobject self, jlong h, jlongArray out) {
    void* p = NULL;
    uint64_t bytes = 0;
    const jint st = zk_deps_partial(CTX(h), &p, &bytes);
    if (st == ZK_OK) {
        const jlong v[2] = {(jlong)(intptr_t)p, (jlong)bytes};
        (*env)->SetLongArrayRegion(env, out, 0, 2, v);
    }
    return st;
}

JNIEXPORT jint JNICALL FN(depsNoteMerged)(JNIEnv* env, jobject self, jlong h, jlong totalRecords) {
    return zk_deps_note_merged(CTX(h), (uint64_t)totalRecords);
}

JNIEXPORT jint JNICALL FN(depsAbort)(JNIEnv* env, jobject self, jlong h) { return zk_deps_abort(CTX(h)); }

JNIEXPORT jint JNICALL FN(traceShard)(JNIEnv* env, jobject self, jlong traceId, jint world) {
    return (jint)zk_trace_shard((uint64_t)traceId, (uint32_t)world);
}

/* ---- multi-GPU (zkcomm.h) ------------------------------------------------------------------------- */
JNIEXPORT jbyteArray JNICALL FN(commUniqueId)(JNIEnv* env, jobject self) {
    uint8_t id[ZK_COMM_ID_BYTES];
    if (zk_comm_unique_id(id, sizeof(id)) != ZK_OK) return NULL;
    jbyteArray out = (*env)->NewByteArray(env, ZK_COMM_ID_BYTES);
    if (out) (*env)->SetByteArrayRegion(env, out, 0, ZK_COMM_ID_BYTES, (const jbyte*)id);
    return out;
}

JNIEXPORT jlong JNICALL FN(commCreate)(JNIEnv* env, jobject self, jbyteArray id, jint rank, jint world, jint dev) {
    if ((*env)->GetArrayLength(env, id) < ZK_COMM_ID_BYTES) return 0;
    uint8_t raw[ZK_COMM_ID_BYTES];
    (*env)->GetByteArrayRegion(env, id, 0, ZK_COMM_ID_BYTES, (jbyte*)raw);
    zk_comm* c = NULL;
    return zk_comm_create(raw, sizeof(raw), (uint32_t)rank, (uint32_t)world, dev, &c) == ZK_OK ? (jlong)(intptr_t)c : 0;
}

JNIEXPORT jint JNICALL FN(commDestroy)(JNIEnv* env, jobject self, jlong comm) { return zk_comm_destroy(COMM(comm)); }

JNIEXPORT jint JNICALL FN(depsAllreduce)(JNIEnv* env, jobject self, jlong h, jlong comm, jlong totalRecords) {
    return zk_deps_allreduce(CTX(h), COMM(comm), (uint64_t)totalRecords);
}

/* ---- realtime link store (zksketch.h zk_rl_*, behind RealtimeAggregates) ---------------------------- */
JNIEXPORT jlong JNICALL FN(rlCreate)(JNIEnv* env, jobject self, jint S, jint dev) {
    zk_rl_config c;
    zk_rl* h = NULL;
    memset(&c, 0, sizeof(c));
    c.num_services = (uint32_t)S;
    c.device = dev;
    return zk_rl_create(&c, &h) == ZK_OK ? (jlong)(intptr_t)h : 0;
}

JNIEXPORT jint JNICALL FN(rlDestroy)(JNIEnv* env, jobject self, jlong rl) { return zk_rl_destroy(RL(rl)); }

JNIEXPORT jint JNICALL FN(rlReset)(JNIEnv* env, jobject self, jlong rl) { return zk_rl_reset(RL(rl)); }

JNIEXPORT jint JNICALL FN(rlBind)(JNIEnv* env, jobject self, jlong h, jlong rl) { return zk_rl_bind(CTX(h), RL(rl)); }

JNIEXPORT jstring JNICALL FN(rlLastError)(JNIEnv* env, jobject self, jlong rl) {
    return (*env)->NewStringUTF(env, zk_rl_last_error(RL(rl)));
}

/* the server's rows as 3 longs each (parent, duration, traceId), ordered by (parent, duration,
   traceId); null on error */
JNIEXPORT jlongArray JNICALL FN(rlServerLinks)(JNIEnv* env, jobject self, jlong rl, jint server) {
    uint64_t n = 0;
    if (zk_rl_server_links(RL(rl), (uint32_t)server, NULL, NULL, NULL, 0, &n) != ZK_OK) return NULL;
    uint32_t* par = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
    int64_t* dur = (int64_t*)malloc((n ? n : 1) * sizeof(int64_t));
    uint64_t* tid = (uint64_t*)malloc((n ? n : 1) * sizeof(uint64_t));
    jlongArray out = NULL;
    if (par && dur && tid && (n == 0 || zk_rl_server_links(RL(rl), (uint32_t)server, par, dur, tid, n, &n) == ZK_OK)) {
        out = (*env)->NewLongArray(env, (jsize)(3 * n));
        for (uint64_t i = 0; out && i < n; ++i) {
            const jlong row[3] = {(jlong)par[i], (jlong)dur[i], (jlong)tid[i]};
            (*env)->SetLongArrayRegion(env, out, (jsize)(3 * i), 3, row);
        }
    }
    free(par);
    free(dur);
    free(tid);
    return out;
}

/* ---- ingest --------------------------------------------------------------------------------------- */
JNIEXPORT jlong JNICALL FN(ingestCreate)(JNIEnv* env, jobject self) {
    zk_ingest* g = NULL;
    return zk_ingest_create(&g) == ZK_OK ? (jlong)(intptr_t)g : 0;
}

JNIEXPORT jint JNICALL FN(ingestDestroy)(JNIEnv* env, jobject self, jlong h) { return zk_ingest_destroy(ING(h)); }

JNIEXPORT jlong JNICALL FN(ingestDecode)(JNIEnv* env, jobject self, jlong h, jobject values, jlongArray offsets,
                                        jint n, jboolean strict, jobject tid, jobject sid, jobject pid, jobject fts,
                                        jobject lts, jobject svc, jobject flg, jlongArray rej) {
    zk_span_cols cols = {BUF(tid), BUF(sid), BUF(pid), BUF(fts), BUF(lts), BUF(svc), BUF(flg), (uint64_t)n};
    jlong* off = (*env)->GetLongArrayElements(env, offsets, NULL);
    uint64_t n_out = 0, n_rej = 0;
    const zk_status st = zk_ingest_spans(ING(h), (const uint8_t*)BUF(values), (const uint64_t*)off, (uint64_t)n,
                                         ZK_CODEC_SNAPPY_THRIFT, strict ? ZK_INGEST_STRICT : 0u, &cols, &n_out,
                                         &n_rej, NULL);
    (*env)->ReleaseLongArrayElements(env, offsets, off, JNI_ABORT);
    const jlong r = (jlong)n_rej;
    (*env)->SetLongArrayRegion(env, rej, 0, 1, &r);
    return st == ZK_OK ? (jlong)n_out : -(jlong)st;
}

JNIEXPORT jint JNICALL FN(ingestNumServices)(JNIEnv* env, jobject self, jlong h) {
    uint32_t n = 0;
    return zk_ingest_num_services(ING(h), &n) == ZK_OK ? (jint)n : -1;
}

JNIEXPORT jstring JNICALL FN(ingestServiceName)(JNIEnv* env, jobject self, jlong h, jint id) {
    uint64_t len = 0;
    if (zk_ingest_service_name(ING(h), (uint32_t)id, NULL, 0, &len) != ZK_OK) return NULL;
    char* buf = (char*)malloc(len + 1);
    if (!buf) return NULL;
    zk_ingest_service_name(ING(h), (uint32_t)id, buf, len, &len);
    buf[len] = 0;
    jstring s = (*env)->NewStringUTF(env, buf);
    free(buf);
    return s;
}

JNIEXPORT jint JNICALL FN(ingestServiceId)(JNIEnv* env, jobject self, jlong h, jstring name) {
    const char* c = (*env)->GetStringUTFChars(env, name, NULL);
    uint32_t id = 0;
    const zk_status st = zk_ingest_service_id(ING(h), c, (uint64_t)strlen(c), &id);
    (*env)->ReleaseStringUTFChars(env, name, c);
    return st == ZK_OK ? (jint)id : -1;
}

/* ---- store ------------------------------------------------------------------------------------------ */
JNIEXPORT jlong JNICALL FN(storeCreate)(JNIEnv* env, jobject self, jint mode) {
    zk_store* s = NULL;
    return zk_store_create((uint32_t)mode, &s) == ZK_OK ? (jlong)(intptr_t)s : 0;
}

JNIEXPORT jint JNICALL FN(storeDestroy)(JNIEnv* env, jobject self, jlong h) { return zk_store_destroy(STORE(h)); }

/* zk_dep_link is 48 bytes: {u32 parent, u32 child, i64 m0, f64 m1..m4} = 6 jlongs, same bit layout */
JNIEXPORT jint JNICALL FN(storePutDependencies)(JNIEnv* env, jobject self, jlong h, jlong startUs, jlong endUs,
                                               jlongArray links) {
    const jsize n = (*env)->GetArrayLength(env, links) / 6;
    jlong* a = (*env)->GetLongArrayElements(env, links, NULL);
    const jint st = zk_store_put_dependencies(STORE(h), startUs, endUs, (const zk_dep_link*)a, (uint64_t)n);
    (*env)->ReleaseLongArrayElements(env, links, a, JNI_ABORT);
    return st;
}

JNIEXPORT jlongArray JNICALL FN(storeGetDependencies)(JNIEnv* env, jobject self, jlong h, jboolean hasStart,
                                                     jlong startUs, jboolean hasEnd, jlong endUs, jlong nowUs,
                                                     jlongArray times) {
    int64_t s = startUs, e = endUs, rs = 0, re = 0;
    uint64_t n = 0;
    const int64_t* ps = hasStart ? &s : NULL;
    const int64_t* pe = hasEnd ? &e : NULL;
    if (zk_store_get_dependencies(STORE(h), ps, pe, nowUs, NULL, 0, &n, &rs, &re) != ZK_OK) return NULL;
    jlongArray out = (*env)->NewLongArray(env, (jsize)(6 * n));
    if (!out) return NULL;
    if (n) {
        jlong* a = (*env)->GetLongArrayElements(env, out, NULL);
        const zk_status st = zk_store_get_dependencies(STORE(h), ps, pe, nowUs, (zk_dep_link*)a, n, &n, &rs, &re);
        (*env)->ReleaseLongArrayElements(env, out, a, 0);
        if (st != ZK_OK) return NULL;
    }
    const jlong t[2] = {rs, re};
    (*env)->SetLongArrayRegion(env, times, 0, 2, t);
    return out;
}

JNIEXPORT jint JNICALL FN(storePutTop)(JNIEnv* env, jobject self, jlong h, jint kind, jint service, jlongArray ids) {
    const jsize n = (*env)->GetArrayLength(env, ids);
    jlong* a = (*env)->GetLongArrayElements(env, ids, NULL);
    const jint st = zk_store_put_top(STORE(h), (uint32_t)kind, (uint32_t)service, (const uint64_t*)a, (uint64_t)n);
    (*env)->ReleaseLongArrayElements(env, ids, a, JNI_ABORT);
    return st;
}

JNIEXPORT jlongArray JNICALL FN(storeGetTop)(JNIEnv* env, jobject self, jlong h, jint kind, jint service) {
    uint64_t n = 0;
    if (zk_store_get_top(STORE(h), (uint32_t)kind, (uint32_t)service, NULL, 0, &n) != ZK_OK) return NULL;
    jlongArray out = (*env)->NewLongArray(env, (jsize)n);
    if (!out || !n) return out;
    jlong* a = (*env)->GetLongArrayElements(env, out, NULL);
    zk_store_get_top(STORE(h), (uint32_t)kind, (uint32_t)service, (uint64_t*)a, n, &n);
    (*env)->ReleaseLongArrayElements(env, out, a, 0);
    return out;
}
