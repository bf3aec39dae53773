/*
 * The dependency job on the GPU: the compute of ZipkinAggregateJob.scala:20-43 (groupBy(id, traceId)
 * .reduce(mergeSpan) -> filter(isValid) -> join on (parentId, traceId) -> Moments(duration) ->
 * group.sum -> one Dependencies) behind a `--compute gpu` switch next to SpanSourceProvider
 * (ZipkinAggregateJob.scala:48-55). NOT COMPILED HERE (no JVM in the build image).
 *
 * Two feeds:
 *  - `runSpans`: decoded Spans (any order; the device clusters them by traceId), turned into the
 *    48-byte records of include/zkagg.h on the JVM;
 *  - `runStored`: the Cassandra column values as stored (Snappy(TBinaryProtocol(Span)),
 *    CassieSpanStore.scala:52): libzkagg decodes them (zkingest.h) and owns the service dictionary,
 *    so the JVM never decodes a span (the reference decodes each one twice, StorageRecordReader.scala:58
 *    and SpanSource.scala:20-22).
 * Output: Dependencies(Time.epoch, Time.now, links) stored through `aggregates`, or nothing when no
 * link exists (:43-45). Strict mode turns a joined span without a service name into a failure, the
 * reference's None.get (:36-37).
 */
package com.twitter.zipkin.gpu

import java.nio.{ByteBuffer, ByteOrder}

import com.twitter.algebird.Moments
import com.twitter.util.{Future, Time}
import com.twitter.zipkin.Constants
import com.twitter.zipkin.common.{Dependencies, DependencyLink, Service, Span}
import com.twitter.zipkin.storage.Aggregates

class GpuDependenciesJob(aggregates: Aggregates, device: Int = 0, strict: Boolean = true,
                         maxTraceRecords: Int = 0) {

  private[this] def direct(n: Int, width: Int) =
    ByteBuffer.allocateDirect(math.max(1, n) * width).order(ByteOrder.LITTLE_ENDIAN)

  private[this] final class Columns(n: Int) {
    val traceId = direct(n, 8); val spanId = direct(n, 8); val parentId = direct(n, 8)
    val firstTs = direct(n, 8); val lastTs = direct(n, 8); val serviceId = direct(n, 4); val flags = direct(n, 4)
  }

  private[this] def fail(ctx: Long, st: Int): Nothing = {
    val msg = ZkNative.lastError(ctx)
    if (st == ZkNative.ErrNoService) throw new NoSuchElementException(s"None.get: $msg") // the reference's crash
    throw new IllegalStateException(s"zk status $st: $msg")
  }

  /** the record of one stored fragment (SURVEY.md Appendix A.1; zkagg.h ZK_F_*) */
  private[this] def put(c: Columns, s: Span, names: Dictionary): Unit = {
    val ts = s.annotations.map(_.timestamp)
    def host(vals: Seq[String]) =
      s.annotations.find(a => vals.contains(a.value) && a.host.isDefined).flatMap(_.host).map(_.serviceName)
    val server = host(Seq(Constants.ServerRecv, Constants.ServerSend))
    val client = host(Seq(Constants.ClientSend, Constants.ClientRecv))
    var f = 0
    if (s.parentId.isDefined) f |= 1
    if (ts.nonEmpty) f |= 2
    val svc = server.map { n => f |= 8; names.id(n) }.orElse(client.map { n => f |= 4; names.id(n) }).getOrElse(0)
    for ((v, shift) <- Seq(Constants.ClientSend -> 8, Constants.ClientRecv -> 10, Constants.ServerRecv -> 12,
                           Constants.ServerSend -> 14))
      f |= math.min(2, s.annotations.count(_.value == v)) << shift
    c.traceId.putLong(s.traceId); c.spanId.putLong(s.id); c.parentId.putLong(s.parentId.getOrElse(0L))
    c.firstTs.putLong(if (ts.nonEmpty) ts.min else 0L); c.lastTs.putLong(if (ts.nonEmpty) ts.max else 0L)
    c.serviceId.putInt(svc); c.flags.putInt(f)
  }

  private[this] def finish(ctx: Long, names: Int => String, S: Int): Option[Dependencies] = {
    val m0 = new Array[Long](S * S); val m1 = new Array[Double](S * S); val m2 = new Array[Double](S * S)
    val m3 = new Array[Double](S * S); val m4 = new Array[Double](S * S); val present = new Array[Byte](S * S)
    val st = ZkNative.finalizeTable(ctx, m0, m1, m2, m3, m4, present)
    if (st != ZkNative.Ok) fail(ctx, st)
    val links = for (c <- 0 until S * S if present(c) != 0)
      yield DependencyLink(Service(names(c / S)), Service(names(c % S)), Moments(m0(c), m1(c), m2(c), m3(c), m4(c)))
    if (links.isEmpty) None else Some(Dependencies(Time.epoch, Time.now, links)) // :41-42
  }

  private[this] def withCtx[T](S: Int)(body: Long => T): T = {
    val ctx = ZkNative.ctxCreate(math.max(1, S), device, strict, maxTraceRecords)
    require(ctx != 0, "zk_ctx_create failed (no gfx950 device?)")
    try body(ctx) finally ZkNative.ctxDestroy(ctx)
  }

  private[this] def store(d: Option[Dependencies]): Future[Option[Dependencies]] = d match {
    case Some(deps) => aggregates.storeDependencies(deps).map(_ => d)
    case None => Future.value(None)
  }

  /** batches of decoded spans; every batch is checked on the device for split traces */
  def runSpans(batches: Iterator[Seq[Span]]): Future[Option[Dependencies]] = {
    val names = new Dictionary
    val cached = batches.toSeq
    cached.foreach(_.foreach(s => s.serviceName.foreach(names.id)))
    val S = names.size
    val out = withCtx(S) { ctx =>
      for (b <- cached) {
        val c = new Columns(b.size)
        b.foreach(put(c, _, names))
        val st = ZkNative.accumulate(ctx, c.traceId, c.spanId, c.parentId, c.firstTs, c.lastTs, c.serviceId,
          c.flags, b.size, ZkNative.BatchVerifyTraces)
        if (st != ZkNative.Ok) fail(ctx, st)
      }
      finish(ctx, names.name, S)
    }
    store(out)
  }

  /** batches of stored column values (the bytes of the traces column family) */
  def runStored(batches: Iterator[Seq[Array[Byte]]]): Future[Option[Dependencies]] = {
    val ing = ZkNative.ingestCreate()
    try {
      val decoded = batches.map { vals =>
        val buf = direct(vals.map(_.length).sum, 1)
        val offsets = vals.scanLeft(0L)(_ + _.length).toArray
        vals.foreach(v => buf.put(v))
        val c = new Columns(vals.size)
        val rejected = new Array[Long](1)
        val n = ZkNative.ingestDecode(ing, buf, offsets, vals.size, strict, c.traceId, c.spanId, c.parentId,
          c.firstTs, c.lastTs, c.serviceId, c.flags, rejected)
        if (n < 0) throw new IllegalArgumentException(s"undecodable span (zk status ${-n})") // thrift.scala:64-121
        (c, n)
      }.toVector
      val S = ZkNative.ingestNumServices(ing)
      val out = withCtx(S) { ctx =>
        for ((c, n) <- decoded) {
          val st = ZkNative.accumulate(ctx, c.traceId, c.spanId, c.parentId, c.firstTs, c.lastTs, c.serviceId,
            c.flags, n, ZkNative.BatchVerifyTraces)
          if (st != ZkNative.Ok) fail(ctx, st)
        }
        finish(ctx, i => ZkNative.ingestServiceName(ing, i), S)
      }
      store(out)
    } finally ZkNative.ingestDestroy(ing)
  }
}
