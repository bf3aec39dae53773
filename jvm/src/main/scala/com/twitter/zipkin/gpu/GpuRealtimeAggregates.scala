/*
 * GpuRealtimeAggregates: the reference's RealtimeAggregates trait (zipkin-common/src/main/scala/com/
 * twitter/zipkin/storage/RealtimeAggregates.scala:26-38), which the reference only implements as
 * NullRealtimeAggregates, backed by libzkagg's realtime link store (include/zksketch.h zk_rl_*).
 * Configured where ThriftQueryService takes `realtimeStore` (ZipkinQueryServerFactory.scala:35,42;
 * ThriftQueryService.scala:317-335 forwards the two queries). NOT COMPILED HERE (no JVM in the build
 * image); zipkin_amd/aggregates.py GpuRealtimeAggregates is its tested twin.
 *
 * The trait's lists (zipkinQuery.thrift:234-251: for a server service, every client service calling
 * it with every span duration / every trace id of those calls) are the dependency job's join rows
 * before its group.sum (ZipkinAggregateJob.scala:25-37): parent span's service = client, child
 * span's service = server, the child span's duration, the trace id. `accumulate(spans, timestamp)`
 * runs the device join over a batch of whole traces (any order) into the time window holding the
 * timestamp; K1 writes the join rows into that window's store beside its links. A query reads the
 * window holding `timeStamp`:
 *   getSpanDurations          Map(client -> every call's duration in us, ascending)
 *   getServiceNamesToTraceIds Map(client -> the calls' distinct trace ids, ascending)
 * and an unknown window or server name gives an empty map, as NullRealtimeAggregates does.
 * rpcName is not a key: the 48-B record carries no span name (the dependency job never reads one),
 * so both cover every rpc of the server; the web UI passes spanName.getOrElse("")
 * (Handlers.scala:83-104). `services` numbers the services (the device keys rows by id); a span naming
 * a service outside it fails its batch.
 */
package com.twitter.zipkin.gpu

import com.twitter.util.{Future, FuturePool, Time}
import com.twitter.zipkin.common.Span
import com.twitter.zipkin.storage.RealtimeAggregates

import scala.collection.mutable

import SpanRecords.{Columns, put}

class GpuRealtimeAggregates(
  services: Seq[String],
  windowUs: Long = 3600L * 1000 * 1000,
  keep: Int = 24,
  device: Int = 0,
  pool: FuturePool = FuturePool.unboundedPool
) extends RealtimeAggregates {
  require(services.nonEmpty && windowUs > 0 && keep > 0)
  private[this] val names = new Dictionary
  services.foreach(names.id)
  private[this] val S = services.size

  /** one time window: a dependency ctx with a link store bound (K1 writes the join rows into it) */
  private[this] final class Window {
    val ctx = ZkNative.ctxCreate(S, device, false, 0)
    require(ctx != 0, "zk_ctx_create failed")
    val rl = ZkNative.rlCreate(S, device)
    require(rl != 0, "zk_rl_create failed")
    check(ZkNative.rlBind(ctx, rl), "zk_rl_bind")
    def close(): Unit = { ZkNative.rlBind(ctx, 0L); ZkNative.rlDestroy(rl); ZkNative.ctxDestroy(ctx) }
  }

  private[this] val windows = mutable.TreeMap.empty[Long, Window]

  private[this] def check(st: Int, what: String): Unit =
    if (st != ZkNative.Ok) throw new IllegalStateException(s"$what: zk status $st")

  private[this] def window(ts: Long, create: Boolean): Option[Window] = synchronized {
    val w = Math.floorDiv(ts, windowUs)
    windows.get(w).orElse {
      if (!create) None
      else {
        val win = new Window
        windows(w) = win
        while (windows.size > keep) { val (k, old) = windows.head; old.close(); windows -= k }
        Some(win)
      }
    }
  }

  /** one batch of whole traces, its spans in any order, into the window of timestampUs */
  def accumulate(spans: Seq[Span], timestampUs: Long): Future[Unit] = pool {
    val c = new Columns(spans.size)
    spans.foreach(put(c, _, names))
    require(names.size == S, "a span names a service outside the store's list")
    val win = window(timestampUs, create = true).get
    win.synchronized {
      check(ZkNative.accumulate(win.ctx, c.traceId, c.spanId, c.parentId, c.firstTs, c.lastTs, c.serviceId, c.flags,
        spans.size, 0), "zk_deps_accumulate")
    }
  }

  /** the server's rows (parent, duration, traceId) in the window of ts, or None */
  private[this] def rows(ts: Time, server: String): Option[Array[Long]] = {
    val id = services.indexOf(server)
    if (id < 0) None
    else window(ts.inMicroseconds, create = false).map { win =>
      win.synchronized {
        val r = ZkNative.rlServerLinks(win.rl, id)
        if (r == null) throw new IllegalStateException(s"zk_rl_server_links: ${ZkNative.rlLastError(win.rl)}")
        r
      }
    }
  }

  def getSpanDurations(timeStamp: Time, serverServiceName: String, rpcName: String): Future[Map[String, List[Long]]] =
    pool {
      rows(timeStamp, serverServiceName) match {
        case None => Map.empty[String, List[Long]]
        case Some(r) =>
          // rows come ordered by (parent, duration): each client's list is ascending already
          (0 until r.length / 3).groupBy(i => r(3 * i).toInt).map { case (p, is) =>
            names.name(p) -> is.map(i => r(3 * i + 1)).toList
          }
      }
    }

  def getServiceNamesToTraceIds(timeStamp: Time, serverServiceName: String, rpcName: String): Future[Map[String, List[Long]]] =
    pool {
      rows(timeStamp, serverServiceName) match {
        case None => Map.empty[String, List[Long]]
        case Some(r) =>
          (0 until r.length / 3).groupBy(i => r(3 * i).toInt).map { case (p, is) =>
            names.name(p) -> is.map(i => r(3 * i + 2)).distinct.sorted.toList
          }
      }
    }

  def close(deadline: Time): Future[Unit] = closeAwaitably {
    synchronized { windows.values.foreach(_.close()); windows.clear() }
    Future.Done
  }
}
