/*
 * JNI surface of libzkagg (include/zkagg.h, zkstore.h, zkingest.h) for the Scala host.
 *
 * NOT COMPILED IN THIS REPOSITORY: the build image has no JVM, Scala or jni.h (SURVEY.md §8c). The
 * natives are implemented by ../c/zkagg_jni.c, which forwards each call to the C ABI unchanged;
 * tests/test_abi.py checks that every zk_* function that file calls is declared in include/*.h.
 * Status codes are returned as Int (0 = ZK_OK); GpuAggregates / GpuDependenciesJob turn non-zero
 * codes into failed Futures, the reference's error convention (QueryService.scala:437-450).
 */
package com.twitter.zipkin.gpu

import java.nio.ByteBuffer

object ZkNative {
  System.loadLibrary("zkagg_jni") // libzkagg_jni.so, linked against libzkagg.so

  final val Ok = 0
  final val ErrNoService = 3
  final val ErrNotClustered = 7
  final val ErrTraceTooLarge = 5
  final val ErrRankFailed = 12
  // zk_deps_accumulate batch flags
  final val BatchDevicePtrs = 1
  final val BatchTraceClustered = 2
  final val BatchContinues = 8  // ZK_BATCH_CONTINUES: the batch's last trace may continue in the next call
  final val BatchVerifyTraces = 4
  // zk_store_create modes
  final val StoreAnorm = 0
  final val StoreCassandra = 1
  final val StoreHBase = 2
  final val TopAnnotations = 0
  final val TopKeyValueAnnotations = 1

  // ---- dependency job (zkagg.h) ----------------------------------------------------------------
  /** zk_ctx_create; returns the handle or 0 (lastError(0) is then meaningless: the status is lost) */
  @native def ctxCreate(numServices: Int, device: Int, strict: Boolean, maxTraceRecords: Int): Long
  @native def ctxDestroy(ctx: Long): Int
  @native def lastError(ctx: Long): String
  @native def reset(ctx: Long): Int
  /** seven direct little-endian ByteBuffers of n records each (host memory, staged over PCIe) */
  @native def accumulate(ctx: Long, traceId: ByteBuffer, spanId: ByteBuffer, parentId: ByteBuffer,
                         firstTs: ByteBuffer, lastTs: ByteBuffer, serviceId: ByteBuffer, flags: ByteBuffer,
                         n: Long, batchFlags: Int): Int
  /** zk_deps_finalize into S*S arrays (cell parent*S + child) */
  @native def finalizeTable(ctx: Long, m0: Array[Long], m1: Array[Double], m2: Array[Double],
                            m3: Array[Double], m4: Array[Double], present: Array[Byte]): Int
  /** zk_ctx_stats: the zk_stats fields in declaration order */
  @native def stats(ctx: Long, out: Array[Long]): Int
  /** zk_deps_partial: out(0) = device pointer of the exchange buffer, out(1) = its bytes (for a host
    * that runs its own int64 SUM all-reduce; depsAllreduce below does it with RCCL) */
  @native def depsPartial(ctx: Long, out: Array[Long]): Int
  @native def depsNoteMerged(ctx: Long, totalRecords: Long): Int
  /** zk_deps_abort: this rank failed before the exchange; after the all-reduce every rank's finalize
    * returns ErrRankFailed (so no rank is left waiting in the collective) */
  @native def depsAbort(ctx: Long): Int
  /** zk_trace_shard: the rank that owns a traceId in a job of `world` ranks */
  @native def traceShard(traceId: Long, world: Int): Int

  // ---- multi-GPU (zkcomm.h): one process per GPU, RCCL over xGMI ---------------------------------
  /** ZK_COMM_ID_BYTES bytes; rank 0 makes it and ships it to the other ranks; null on error */
  @native def commUniqueId(): Array[Byte]
  /** blocks until all `world` ranks joined; 0 on error */
  @native def commCreate(id: Array[Byte], rank: Int, world: Int, device: Int): Long
  @native def commDestroy(comm: Long): Int
  /** zk_deps_partial -> RCCL int64 SUM of the exchange buffer -> zk_deps_note_merged (0 = total from
    * the merged counters) */
  @native def depsAllreduce(ctx: Long, comm: Long, totalRecords: Long): Int

  // ---- realtime link store (zksketch.h zk_rl_*): the state behind GpuRealtimeAggregates -----------
  /** 0 on error */
  @native def rlCreate(numServices: Int, device: Int): Long
  @native def rlDestroy(rl: Long): Int
  @native def rlReset(rl: Long): Int
  /** K1 of every later accumulate on ctx writes its join rows into rl (rl = 0 unbinds) */
  @native def rlBind(ctx: Long, rl: Long): Int
  @native def rlLastError(rl: Long): String
  /** the rows whose child (server) service is `server`: (parent, duration us, traceId) triples ordered
    * by (parent, duration, traceId); null on error */
  @native def rlServerLinks(rl: Long, server: Int): Array[Long]

  // ---- ingest (zkingest.h) -----------------------------------------------------------------------
  @native def ingestCreate(): Long
  @native def ingestDestroy(ing: Long): Int
  /** stored Cassandra column values back to back; returns records written or -(status) */
  @native def ingestDecode(ing: Long, values: ByteBuffer, offsets: Array[Long], n: Int, strict: Boolean,
                           traceId: ByteBuffer, spanId: ByteBuffer, parentId: ByteBuffer, firstTs: ByteBuffer,
                           lastTs: ByteBuffer, serviceId: ByteBuffer, flags: ByteBuffer,
                           rejected: Array[Long]): Long
  @native def ingestNumServices(ing: Long): Int
  @native def ingestServiceName(ing: Long, id: Int): String
  @native def ingestServiceId(ing: Long, name: String): Int

  // ---- store (zkstore.h) ---------------------------------------------------------------------------
  @native def storeCreate(mode: Int): Long
  @native def storeDestroy(store: Long): Int
  /** links: zk_dep_link as 6 longs each (parent | child << 32, m0, m1..m4 as raw double bits) */
  @native def storePutDependencies(store: Long, startUs: Long, endUs: Long, links: Array[Long]): Int
  /** returns the links in the same 6-long layout; times(0..1) receive the result's start/end (us);
    * null on error */
  @native def storeGetDependencies(store: Long, hasStart: Boolean, startUs: Long, hasEnd: Boolean, endUs: Long,
                                   nowUs: Long, times: Array[Long]): Array[Long]
  @native def storePutTop(store: Long, kind: Int, service: Int, ids: Array[Long]): Int
  @native def storeGetTop(store: Long, kind: Int, service: Int): Array[Long]
}
