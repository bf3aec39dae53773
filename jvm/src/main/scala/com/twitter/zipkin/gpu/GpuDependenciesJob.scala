/*
 * The dependency job on the GPU: the compute of ZipkinAggregateJob.scala:20-43 (groupBy(id, traceId)
 * .reduce(mergeSpan) -> filter(isValid) -> join on (parentId, traceId) -> Moments(duration) ->
 * group.sum -> one Dependencies) behind a `--compute gpu` switch next to SpanSourceProvider
 * (ZipkinAggregateJob.scala:48-55). NOT COMPILED HERE (no JVM in the build image).
 *
 * Two feeds, both streamed batch by batch (nothing is materialised beyond two batches):
 *  - `runStored`: the Cassandra column values as stored (Snappy(TBinaryProtocol(Span)),
 *    CassieSpanStore.scala:52), in the order a row-per-trace reader returns them
 *    (StorageRecordReader.scala:49-54): every trace's fragments are adjacent, and a batch may end in
 *    the middle of a trace. libzkagg decodes them (zkingest.h) and owns the service dictionary, so the
 *    JVM never decodes a span (the reference decodes each one twice, StorageRecordReader.scala:58 and
 *    SpanSource.scala:20-22). Batches go in with ZK_BATCH_TRACE_CLUSTERED | ZK_BATCH_CONTINUES -- the
 *    path bench.py measures -- and batch k+1 is decoded on a second thread while batch k accumulates.
 *  - `runSpans`: decoded Spans in any order, each batch holding whole traces; the device clusters
 *    every batch by traceId.
 * `verify` adds ZK_BATCH_VERIFY_TRACES (an exact device check that no trace recurs after its run
 * ended; 16 B of HBM per record).
 *
 * Multi-GPU (`shard`): one JVM process per GPU, each reading a traceId-disjoint part of the input (a
 * split by Cassandra/HBase row key is; other sources keep the spans with
 * ZkNative.traceShard(traceId, world) == rank). After the last batch every rank calls depsAllreduce --
 * one RCCL int64 SUM of the exact table's exchange form, the reference's cross-reducer .group.sum /
 * .sum (:39-43) -- and finalizes the same job-wide table with the same status; rank 0 stores it. A
 * rank that fails on the host before the exchange still makes that call, with an abort mark
 * (`guarded`), so the others fail with ErrRankFailed instead of blocking in RCCL.
 *
 * Output: Dependencies(Time.epoch, Time.now, links) stored through `aggregates`, or nothing when no
 * link exists (:43-45). Strict mode turns a joined span without a service name into a failure, the
 * reference's None.get (:36-37). `numServices` is the capacity of the service dictionary (the
 * S x S device table is sized from it; a service id beyond it fails the job with
 * ZK_ERR_SERVICE_RANGE). `services` seeds the dictionary in a fixed order (e.g. from
 * SpanStore.getAllServiceNames): a multi-GPU job needs it, because the ranks' tables are summed cell
 * by cell and so must agree on every service id -- a rank that meets a name outside the list fails.
 */
package com.twitter.zipkin.gpu

import java.util.concurrent.{Callable, Executors}

import com.twitter.algebird.Moments
import com.twitter.util.{Future, Time}
import com.twitter.zipkin.common.{Dependencies, DependencyLink, Service, Span}
import com.twitter.zipkin.storage.Aggregates

import SpanRecords.{Columns, direct, put}

/** rank / world of a multi-GPU job and the communicator id rank 0 made (ZkNative.commUniqueId) */
final case class GpuShard(rank: Int, world: Int, commId: Array[Byte])

class GpuDependenciesJob(aggregates: Aggregates, device: Int = 0, strict: Boolean = true,
                         maxTraceRecords: Int = 0, numServices: Int = 1024, verify: Boolean = false,
                         services: Seq[String] = Nil, shard: Option[GpuShard] = None) {
  require(shard.isEmpty || services.nonEmpty, "a multi-GPU job needs the service list every rank numbers alike")
  require(services.size <= numServices, "more services than numServices")

  private[this] def fail(ctx: Long, st: Int): Nothing = {
    val msg = ZkNative.lastError(ctx)
    if (st == ZkNative.ErrNoService) throw new NoSuchElementException(s"None.get: $msg") // the reference's crash
    if (st == ZkNative.ErrRankFailed) throw new IllegalStateException(s"another rank of the job failed: $msg")
    throw new IllegalStateException(s"zk status $st: $msg")
  }

  private[this] def check(ctx: Long, st: Int): Unit = if (st != ZkNative.Ok) fail(ctx, st)

  private[this] def accumulate(ctx: Long, c: Columns, n: Long, flags: Int): Unit =
    check(ctx, ZkNative.accumulate(ctx, c.traceId, c.spanId, c.parentId, c.firstTs, c.lastTs, c.serviceId, c.flags,
      n, flags | (if (verify) ZkNative.BatchVerifyTraces else 0)))

  /** [all-reduce across ranks,] finalize; the Dependencies record of the whole job on every rank */
  private[this] def finish(ctx: Long, comm: Long, names: Int => String): Option[Dependencies] = {
    if (comm != 0) check(ctx, ZkNative.depsAllreduce(ctx, comm, 0L))
    val S = numServices
    val m0 = new Array[Long](S * S); val m1 = new Array[Double](S * S); val m2 = new Array[Double](S * S)
    val m3 = new Array[Double](S * S); val m4 = new Array[Double](S * S); val present = new Array[Byte](S * S)
    check(ctx, ZkNative.finalizeTable(ctx, m0, m1, m2, m3, m4, present))
    val links = for (c <- 0 until S * S if present(c) != 0)
      yield DependencyLink(Service(names(c / S)), Service(names(c % S)), Moments(m0(c), m1(c), m2(c), m3(c), m4(c)))
    if (links.isEmpty) None else Some(Dependencies(Time.epoch, Time.now, links)) // :41-42
  }

  private[this] def withCtx[T](body: (Long, Long) => T): T = {
    val ctx = ZkNative.ctxCreate(numServices, device, strict, maxTraceRecords)
    require(ctx != 0, "zk_ctx_create failed (no gfx950 device?)")
    val comm = shard match {
      case Some(GpuShard(rank, world, id)) =>
        val c = ZkNative.commCreate(id, rank, world, device)
        require(c != 0, s"zk_comm_create failed (rank $rank of $world)")
        c
      case None => 0L
    }
    try body(ctx, comm) finally {
      if (comm != 0) ZkNative.commDestroy(comm)
      ZkNative.ctxDestroy(ctx)
    }
  }

  /** the rank's part of the job before the exchange. A rank that fails here on the host (an
    * undecodable span, a refused batch, a service outside the job's list, the decoder thread) still
    * makes the job's one collective call, with an abort mark (zk_deps_abort): every other rank's
    * finalize then fails with ErrRankFailed instead of waiting in the all-reduce forever. */
  private[this] def guarded(ctx: Long, comm: Long)(part: => Unit): Unit =
    try part catch {
      case e: Throwable if comm != 0 =>
        ZkNative.depsAbort(ctx)
        ZkNative.depsAllreduce(ctx, comm, 0L) // (its own status is moot: this rank rethrows)
        throw e
    }

  /** rank 0 stores the job's record (every rank holds the same one) */
  private[this] def store(d: Option[Dependencies]): Future[Option[Dependencies]] = d match {
    case Some(deps) if shard.forall(_.rank == 0) => aggregates.storeDependencies(deps).map(_ => d)
    case _ => Future.value(d)
  }

  /** trace-complete batches of decoded spans in any order; the device clusters each batch by traceId */
  def runSpans(batches: Iterator[Seq[Span]]): Future[Option[Dependencies]] = {
    val names = new Dictionary
    services.foreach(names.id)
    val out = withCtx { (ctx, comm) =>
      guarded(ctx, comm) {
        for (b <- batches) {
          val c = new Columns(b.size)
          b.foreach(put(c, _, names))
          require(names.size <= numServices, s"more than $numServices service names")
          require(shard.isEmpty || names.size == services.size, "a span names a service outside the job's list")
          accumulate(ctx, c, b.size, 0)
        }
      }
      finish(ctx, comm, names.name)
    }
    store(out)
  }

  /** batches of stored column values (the bytes of the traces column family) in row order */
  def runStored(batches: Iterator[Seq[Array[Byte]]]): Future[Option[Dependencies]] = {
    val ing = ZkNative.ingestCreate()
    services.foreach(ZkNative.ingestServiceId(ing, _))  // ids 0..n-1 in the list's order, on every rank
    val decoder = Executors.newSingleThreadExecutor()
    def decode(vals: Seq[Array[Byte]]): (Columns, Long) = {
      val buf = direct(vals.map(_.length).sum, 1)
      val offsets = vals.scanLeft(0L)(_ + _.length).toArray
      vals.foreach(v => buf.put(v))
      val c = new Columns(vals.size)
      val rejected = new Array[Long](1)
      val n = ZkNative.ingestDecode(ing, buf, offsets, vals.size, strict, c.traceId, c.spanId, c.parentId,
        c.firstTs, c.lastTs, c.serviceId, c.flags, rejected)
      if (n < 0) throw new IllegalArgumentException(s"undecodable span (zk status ${-n})") // thrift.scala:64-121
      (c, n)
    }
    def submit(vals: Seq[Array[Byte]]) = decoder.submit(new Callable[(Columns, Long)] { def call() = decode(vals) })
    try {
      val out = withCtx { (ctx, comm) =>
        guarded(ctx, comm) {
          // batch k accumulates (PCIe staging + device work) while batch k+1 decodes on the other thread
          var next = if (batches.hasNext) Some(submit(batches.next())) else None
          while (next.isDefined) {
            val (c, n) = next.get.get()
            next = if (batches.hasNext) Some(submit(batches.next())) else None
            // the reader cuts batches anywhere: the batch's last trace may continue in the next one
            accumulate(ctx, c, n, ZkNative.BatchTraceClustered | ZkNative.BatchContinues)
          }
          val S = ZkNative.ingestNumServices(ing)
          require(S <= numServices, s"$S service names > numServices = $numServices")
          require(shard.isEmpty || S == services.size, "a stored span names a service outside the job's list")
        }
        finish(ctx, comm, i => ZkNative.ingestServiceName(ing, i))
      }
      store(out)
    } finally {
      decoder.shutdownNow()
      ZkNative.ingestDestroy(ing)
    }
  }
}
