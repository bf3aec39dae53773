/*
 * GpuAggregates: the reference's Aggregates trait (zipkin-common/src/main/scala/com/twitter/zipkin/
 * storage/Aggregates.scala:26-37) backed by libzkagg's store (include/zkstore.h) -- a drop-in for
 * the CassandraAggregates / AnormAggregates / HBaseAggregates a query or collector service is
 * configured with (Store.scala:26-38). NOT COMPILED HERE (no JVM in the build image).
 *
 * Strings stay on the JVM: services and annotation strings are interned into dictionary ids, the
 * store sees ids only. Calls run on a FuturePool like AnormAggregates' (AnormThreads.scala:26,31);
 * zk_store is thread-safe (its own lock, the reference's `synchronized`).
 */
package com.twitter.zipkin.gpu

import java.lang.{Double => JDouble}
import java.util.concurrent.ConcurrentHashMap

import com.twitter.algebird.Moments
import com.twitter.util.{Future, FuturePool, Time}
import com.twitter.zipkin.common.{Dependencies, DependencyLink, Service}
import com.twitter.zipkin.storage.Aggregates

import scala.collection.mutable.ArrayBuffer

/** a thread-safe string <-> dense id dictionary (case-sensitive, like Service(name)) */
class Dictionary {
  private[this] val ids = new ConcurrentHashMap[String, Integer]()
  private[this] val names = ArrayBuffer[String]()
  def id(name: String): Int = synchronized {
    val got = ids.get(name)
    if (got != null) got.intValue else { ids.put(name, names.size); names += name; names.size - 1 }
  }
  def name(id: Int): String = synchronized { names(id) }
  def size: Int = synchronized { names.size }
}

class GpuAggregates(
  mode: Int = ZkNative.StoreAnorm,
  val services: Dictionary = new Dictionary,
  val strings: Dictionary = new Dictionary,
  pool: FuturePool = FuturePool.unboundedPool
) extends Aggregates {

  private[this] val store = {
    val h = ZkNative.storeCreate(mode)
    require(h != 0, "zk_store_create failed")
    h
  }

  private[this] def check(st: Int, what: String): Unit =
    if (st != ZkNative.Ok) throw new IllegalStateException(s"$what: zk status $st")

  def close(): Unit = ZkNative.storeDestroy(store)

  def storeDependencies(d: Dependencies): Future[Unit] = pool {
    check(ZkNative.storePutDependencies(store, d.startTime.inMicroseconds, d.endTime.inMicroseconds, pack(d.links)),
      "storeDependencies")
  }

  // zk_dep_link = {u32 parent, u32 child, i64 m0, f64 m1..m4}: 6 x 8 bytes, the first word packs
  // both ids (little-endian: parent in the low half)
  private[this] def pack(links: Seq[DependencyLink]): Array[Long] = {
    val out = new Array[Long](6 * links.size)
    for ((l, i) <- links.zipWithIndex) {
      val m = l.durationMoments
      out(6 * i) = (services.id(l.child.name).toLong << 32) | (services.id(l.parent.name).toLong & 0xFFFFFFFFL)
      out(6 * i + 1) = m.m0
      out(6 * i + 2) = JDouble.doubleToRawLongBits(m.m1)
      out(6 * i + 3) = JDouble.doubleToRawLongBits(m.m2)
      out(6 * i + 4) = JDouble.doubleToRawLongBits(m.m3)
      out(6 * i + 5) = JDouble.doubleToRawLongBits(m.m4)
    }
    out
  }

  def getDependencies(startDate: Option[Time], endDate: Option[Time] = None): Future[Dependencies] = pool {
    val times = new Array[Long](2)
    val a = ZkNative.storeGetDependencies(store, startDate.isDefined, startDate.map(_.inMicroseconds).getOrElse(0L),
      endDate.isDefined, endDate.map(_.inMicroseconds).getOrElse(0L), Time.now.inMicroseconds, times)
    if (a == null) throw new IllegalStateException("getDependencies failed")
    val links = (0 until a.length / 6).map { i =>
      val ids = a(6 * i)
      DependencyLink(Service(services.name((ids & 0xFFFFFFFFL).toInt)), Service(services.name((ids >>> 32).toInt)),
        Moments(a(6 * i + 1), JDouble.longBitsToDouble(a(6 * i + 2)), JDouble.longBitsToDouble(a(6 * i + 3)),
          JDouble.longBitsToDouble(a(6 * i + 4)), JDouble.longBitsToDouble(a(6 * i + 5))))
    }
    // ZK_TIME_TOP / ZK_TIME_BOTTOM are the monoid zero's Time.Top / Time.Bottom
    def time(us: Long) = if (us == Long.MaxValue) Time.Top else if (us == Long.MinValue) Time.Bottom
                         else Time.fromMicroseconds(us)
    Dependencies(time(times(0)), time(times(1)), links)
  }

  private[this] def putTop(kind: Int, serviceName: String, a: Seq[String]): Future[Unit] = pool {
    check(ZkNative.storePutTop(store, kind, services.id(serviceName), a.map(s => strings.id(s).toLong).toArray),
      "storeTop")
  }
  private[this] def getTop(kind: Int, serviceName: String): Future[Seq[String]] = pool {
    val ids = ZkNative.storeGetTop(store, kind, services.id(serviceName))
    if (ids == null) Seq.empty[String] else ids.toSeq.map(i => strings.name(i.toInt))
  }

  def getTopAnnotations(serviceName: String) = getTop(ZkNative.TopAnnotations, serviceName)
  def getTopKeyValueAnnotations(serviceName: String) = getTop(ZkNative.TopKeyValueAnnotations, serviceName)
  def storeTopAnnotations(serviceName: String, a: Seq[String]) = putTop(ZkNative.TopAnnotations, serviceName, a)
  def storeTopKeyValueAnnotations(serviceName: String, a: Seq[String]) =
    putTop(ZkNative.TopKeyValueAnnotations, serviceName, a)
}
