/*
 * The 48-B columnar record of one stored span fragment (include/zkagg.h zk_span_cols, ZK_F_*), built
 * on the JVM from a decoded Span for the calls that take Spans (GpuDependenciesJob.runSpans,
 * GpuRealtimeAggregates.accumulate); the stored-bytes path decodes in libzkagg instead (zkingest.h).
 * NOT COMPILED HERE (no JVM in the build image).
 */
package com.twitter.zipkin.gpu

import java.nio.{ByteBuffer, ByteOrder}

import com.twitter.zipkin.Constants
import com.twitter.zipkin.common.Span

object SpanRecords {
  def direct(n: Int, width: Int): ByteBuffer =
    ByteBuffer.allocateDirect(math.max(1, n) * width).order(ByteOrder.LITTLE_ENDIAN)

  /** seven direct little-endian columns of n records (host memory, staged over PCIe by the library;
    * borrowed for the duration of the accumulate call only, zkagg.h) */
  final class Columns(n: Int) {
    val traceId = direct(n, 8); val spanId = direct(n, 8); val parentId = direct(n, 8)
    val firstTs = direct(n, 8); val lastTs = direct(n, 8); val serviceId = direct(n, 4); val flags = direct(n, 4)
  }

  /** the record of one stored fragment (SURVEY.md Appendix A.1; zkagg.h ZK_F_*) */
  def put(c: Columns, s: Span, names: Dictionary): Unit = {
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
}
