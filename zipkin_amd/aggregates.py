"""Host mirror of the reference's Aggregates surface over libzkagg (include/zkstore.h, zkagg.h).

Same names, argument meaning and error behaviour as
  trait Aggregates            zipkin-common/.../storage/Aggregates.scala:26-37
  class NullAggregates        Aggregates.scala:39-50
  Service / DependencyLink / Dependencies   zipkin-common/.../common/Dependencies.scala:25-83
  algebird Moments            (algebird-core 0.8.1; accessors as zipkin-web momentAnnotations.js:5-19)
and a driver for the job itself (ZipkinAggregateJob.scala:20-45) that runs the device path and hands
its single Dependencies record to `storeDependencies`.

Times are microseconds since the epoch (Time.inMicroseconds, zipkinDependencies.thrift:40-41).
The reference's failed Futures are raised here as ZkError (the C status) or AssertionError
(DependencyLink.sg's key assert, Dependencies.scala:40). Moments arithmetic runs in the library
(zk_moments_plus); nothing here computes on the CPU what the device path produces.
"""
from __future__ import annotations

import ctypes as C
import time
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, NamedTuple, Optional, Sequence

import numpy as np

from . import _abi

DAY_US = 86_400 * 1_000_000


def now_us() -> int:
    return time.time_ns() // 1000


class Moments(NamedTuple):
    """algebird Moments(m0 = count, m1 = mean, m2..m4 = central moment sums)."""

    m0: int
    m1: float
    m2: float
    m3: float
    m4: float

    @staticmethod
    def of(value: float) -> "Moments":  # Moments(value) (ZipkinAggregateJob.scala:35)
        return Moments(1, float(value), 0.0, 0.0, 0.0)

    @staticmethod
    def zero() -> "Moments":
        return Moments(0, 0.0, 0.0, 0.0, 0.0)

    def plus(self, other: "Moments") -> "Moments":
        """MomentsGroup.plus (through zk_moments_plus)."""
        out = _abi.zk_moments()
        st = _abi.lib().zk_moments_plus(C.byref(_to_c(self)), C.byref(_to_c(other)), C.byref(out))
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, _abi.status_str(st))
        return _from_c(out)

    # momentAnnotations.js:6-11
    @property
    def count(self) -> int:
        return self.m0

    @property
    def mean(self) -> float:
        return self.m1

    @property
    def variance(self) -> float:
        return self.m2 / self.m0

    @property
    def stddev(self) -> float:
        return self.variance ** 0.5

    @property
    def skewness(self) -> float:
        return (self.m0 ** 0.5) * self.m3 / (self.m2 ** 1.5)

    @property
    def kurtosis(self) -> float:
        return self.m0 * self.m4 / (self.m2 ** 2) - 3


def _to_c(m: Moments) -> "_abi.zk_moments":
    return _abi.zk_moments(int(m.m0), float(m.m1), float(m.m2), float(m.m3), float(m.m4))


def _from_c(m) -> Moments:
    return Moments(int(m.m0), float(m.m1), float(m.m2), float(m.m3), float(m.m4))


@dataclass(frozen=True)
class Service:
    name: str  # case-sensitive (DependenciesTest.scala:28-40)


@dataclass(frozen=True)
class DependencyLink:
    parent: Service
    child: Service
    duration_moments: Moments

    def plus(self, r: "DependencyLink") -> "DependencyLink":
        """DependencyLink.sg.plus (Dependencies.scala:38-43)."""
        assert self.child == r.child and self.parent == r.parent
        return DependencyLink(self.parent, self.child, self.duration_moments.plus(r.duration_moments))


@dataclass(frozen=True)
class Dependencies:
    start_time: int
    end_time: int
    links: tuple = field(default_factory=tuple)

    @staticmethod
    def zero() -> "Dependencies":  # Dependencies.scala:81 (Time.Top, Time.Bottom)
        return Dependencies(_abi.ZK_TIME_TOP, _abi.ZK_TIME_BOTTOM, ())

    def plus(self, r: "Dependencies") -> "Dependencies":
        """Dependencies.monoid.plus(l = self, r) (Dependencies.scala:68-79)."""
        lmap = {(l.parent, l.child): l for l in self.links}
        rmap = {(l.parent, l.child): l for l in r.links}
        merged = dict(rmap)
        for k, l in lmap.items():  # Monoid.plus(rLinkMap, lLinkMap): sg.plus(r, l) on shared keys
            merged[k] = merged[k].plus(l) if k in merged else l
        return Dependencies(min(r.start_time, self.start_time), max(r.end_time, self.end_time),
                            tuple(merged.values()))


_DEP_LINK_DTYPE = np.dtype([("parent", "<u4"), ("child", "<u4"), ("m0", "<i8"), ("m1", "<f8"), ("m2", "<f8"),
                            ("m3", "<f8"), ("m4", "<f8")])  # zk_dep_link (zkstore.h), 48 B


class LinkList:
    """The links of a Dependencies record kept in the job's finalized form until read: the dense
    host table (present cells = links) and the service names of its ids. The compact zk_dep_link
    array (zk_link_table_compact, cell order) is built on first use, the DependencyLink objects on
    first iteration -- so a job over 10^5 (parent, child) pairs returns its record without 10^5 Python
    objects, and storeDependencies passes the compact array to the store as it is."""

    def __init__(self, table, names: List[str]):
        self._table, self._names = table, names
        self._raw = self._items = None
        self._n = int(np.count_nonzero(table.present))

    def compact(self):
        """(zk_dep_link structured array, names of its ids)."""
        if self._raw is None:
            t = self._table
            ct = _abi.zk_link_table()
            ct.m0, ct.m1, ct.m2, ct.m3, ct.m4 = (a.ctypes.data for a in (t.m0, t.m1, t.m2, t.m3, t.m4))
            ct.present = t.present.ctypes.data
            ct.device_ptrs = 0
            raw = np.empty(max(self._n, 1), _DEP_LINK_DTYPE)
            n = C.c_uint64()
            st = _abi.lib().zk_link_table_compact(C.byref(ct), t.num_services, raw.ctypes.data, self._n, C.byref(n))
            if st != _abi.ZK_OK:
                raise _abi.ZkError(st, _abi.status_str(st))
            self._raw = raw[: n.value]
        return self._raw, self._names

    def _all(self) -> tuple:
        if self._items is None:
            nm, r = self._names, self.compact()[0]
            self._items = tuple(
                DependencyLink(Service(nm[int(p)]), Service(nm[int(c)]), Moments(int(m0), float(a), float(b), float(x),
                                                                                  float(y)))
                for p, c, m0, a, b, x, y in zip(r["parent"], r["child"], r["m0"], r["m1"], r["m2"], r["m3"], r["m4"]))
        return self._items

    def __len__(self):
        return self._n

    def __iter__(self):
        return iter(self._all())

    def __getitem__(self, i):
        return self._all()[i]

    def __eq__(self, other):
        return tuple(self._all()) == tuple(other)

    def __ne__(self, other):
        return not self == other

    def __hash__(self):
        return hash(self._all())

    def __repr__(self):
        return repr(self._all())


class Dictionary:
    """Host-owned string <-> id dictionary (service names, annotation values / keys)."""

    def __init__(self, names: Iterable[str] = ()):
        self._ids: Dict[str, int] = {}
        self._names: List[str] = []
        for n in names:
            self.id(n)

    def id(self, name: str) -> int:
        i = self._ids.get(name)
        if i is None:
            i = len(self._names)
            self._ids[name] = i
            self._names.append(name)
        return i

    def get(self, name: str) -> Optional[int]:
        return self._ids.get(name)

    def name(self, i: int) -> str:
        return self._names[i]

    def __len__(self) -> int:
        return len(self._names)

    def __contains__(self, name: str) -> bool:
        return name in self._ids


class Aggregates:
    """trait Aggregates (Aggregates.scala:26-37)."""

    def close(self) -> None:
        raise NotImplementedError

    def getDependencies(self, startDate: Optional[int], endDate: Optional[int] = None) -> Dependencies:
        raise NotImplementedError

    def storeDependencies(self, dependencies: Dependencies) -> None:
        raise NotImplementedError

    def getTopAnnotations(self, serviceName: str) -> List[str]:
        raise NotImplementedError

    def getTopKeyValueAnnotations(self, serviceName: str) -> List[str]:
        raise NotImplementedError

    def storeTopAnnotations(self, serviceName: str, a: Sequence[str]) -> None:
        raise NotImplementedError

    def storeTopKeyValueAnnotations(self, serviceName: str, a: Sequence[str]) -> None:
        raise NotImplementedError


class NullAggregates(Aggregates):
    """NullAggregates (Aggregates.scala:39-50)."""

    def close(self) -> None:
        pass

    def getDependencies(self, startDate=None, endDate=None) -> Dependencies:
        return Dependencies.zero()

    def storeDependencies(self, dependencies) -> None:
        pass

    def getTopAnnotations(self, serviceName) -> List[str]:
        return []

    def getTopKeyValueAnnotations(self, serviceName) -> List[str]:
        return []

    def storeTopAnnotations(self, serviceName, a) -> None:
        pass

    def storeTopKeyValueAnnotations(self, serviceName, a) -> None:
        pass


class RealtimeAggregates:
    """trait RealtimeAggregates (zipkin-common/.../storage/RealtimeAggregates.scala:26-38): for a
    time stamp (us), a server service name and an rpc name, a map from every client service calling
    that server to a list -- of every span duration (getSpanDurations) or every trace id
    (getServiceNamesToTraceIds) of those calls (zipkinQuery.thrift:234-251)."""

    def close(self) -> None:
        raise NotImplementedError

    def getSpanDurations(self, timeStamp: int, serverServiceName: str, rpcName: str) -> Dict[str, List[int]]:
        raise NotImplementedError

    def getServiceNamesToTraceIds(self, timeStamp: int, serverServiceName: str, rpcName: str) -> Dict[str, List[int]]:
        raise NotImplementedError


class NullRealtimeAggregates(RealtimeAggregates):
    """NullRealtimeAggregates (RealtimeAggregates.scala:40-51): empty maps."""

    def close(self) -> None:
        pass

    def getSpanDurations(self, timeStamp, serverServiceName, rpcName) -> Dict[str, List[int]]:
        return {}

    def getServiceNamesToTraceIds(self, timeStamp, serverServiceName, rpcName) -> Dict[str, List[int]]:
        return {}


def _signed64(x: int) -> int:
    """a traceId as the JVM's Long (zipkinQuery.thrift i64)"""
    return x - (1 << 64) if x >= 1 << 63 else x


class _DeviceLinkWindow:
    """One time window of GpuRealtimeAggregates on the device: a DepsContext with a RealtimeLinks
    store bound (K1 writes the join rows beside its links)."""

    def __init__(self, num_services: int, device: int):
        from .context import DepsContext
        from .realtime import RealtimeLinks

        self.ctx = DepsContext(num_services, device=device, strict=False)
        self.rl = RealtimeLinks(num_services, device=device)
        self.rl.bind(self.ctx)

    def add(self, cols, clustered: bool) -> None:
        self.ctx.accumulate(cols, clustered=clustered, verify=False)

    def server_links(self, server: int):
        self.ctx.sync()
        return self.rl.server_links(server)

    def close(self) -> None:
        self.rl.close()
        self.ctx.close()


class GpuRealtimeAggregates(RealtimeAggregates):
    """RealtimeAggregates over the device's join rows (include/zksketch.h zk_rl_*).

    The rows the trait's lists are made of are the dependency job's join rows before its group.sum
    (ZipkinAggregateJob.scala:25-37): parent span's service = the CLIENT service, child span's
    service = the SERVER service, the child span's duration, the trace id. `accumulate(batch,
    timestamp)` runs the device join over a batch of span fragments (any order; whole traces per
    batch) into the time window holding `timestamp` (windows of `window_us`, the last `keep` kept);
    the queries answer from the window holding `timeStamp` (Time in us, ThriftQueryService.scala:317-
    335), with an empty map for an unknown window or server name:

      getSpanDurations(t, server, rpc)          {client: every call's duration in us, ascending}
      getServiceNamesToTraceIds(t, server, rpc) {client: the calls' distinct trace ids, ascending,
                                                 as signed 64-bit Longs}

    rpcName is not a key: the 48-B record carries no span name (the dependency job never reads
    one), so both answers cover every rpc of the server; the web UI passes spanName.getOrElse("")
    (Handlers.scala:83-104). `window_factory(num_services)` builds a window (default: the device);
    the CPU tests pass the oracle's."""

    def __init__(self, services: Dictionary, *, window_us: int = 3_600_000_000, keep: int = 24, device: int = 0,
                 window_factory=None):
        if window_us <= 0 or keep <= 0:
            raise ValueError("window_us and keep must be positive")
        self.services = services
        self.window_us = int(window_us)
        self.keep = int(keep)
        self._factory = window_factory or (lambda S: _DeviceLinkWindow(S, device))
        self._windows: Dict[int, object] = {}

    def _window(self, timestamp_us: int, create: bool):
        w = int(timestamp_us) // self.window_us
        win = self._windows.get(w)
        if win is None and create:
            win = self._factory(max(1, len(self.services)))
            self._windows[w] = win
            for old in sorted(self._windows)[:-self.keep]:  # the oldest windows leave the store
                self._windows.pop(old).close()
        return win

    def accumulate(self, cols, timestamp_us: int, *, clustered: bool = False) -> None:
        """One batch of span fragments (service ids from `services`) into the window of timestamp_us."""
        self._window(timestamp_us, True).add(cols, clustered)

    def _rows(self, timeStamp: int, serverServiceName: str):
        win = self._window(timeStamp, False)
        if win is None or serverServiceName not in self.services:
            return None
        return win.server_links(self.services.id(serverServiceName))

    def getSpanDurations(self, timeStamp: int, serverServiceName: str, rpcName: str) -> Dict[str, List[int]]:
        rows = self._rows(timeStamp, serverServiceName)
        if rows is None:
            return {}
        par, dur, _ = rows
        out: Dict[str, List[int]] = {}
        for p, d in zip(par.tolist(), dur.tolist()):  # (rows come ordered by parent, then duration)
            out.setdefault(self.services.name(p), []).append(int(d))
        return out

    def getServiceNamesToTraceIds(self, timeStamp: int, serverServiceName: str, rpcName: str) -> Dict[str, List[int]]:
        rows = self._rows(timeStamp, serverServiceName)
        if rows is None:
            return {}
        par, _, tid = rows
        out: Dict[str, set] = {}
        for p, t in zip(par.tolist(), tid.tolist()):
            out.setdefault(self.services.name(p), set()).add(int(t))
        return {k: sorted(_signed64(t) for t in v) for k, v in out.items()}

    def close(self) -> None:
        for win in self._windows.values():
            win.close()
        self._windows = {}


class GpuAggregates(Aggregates):
    """Aggregates over a zk_store with one reference backend's storage semantics (zkstore.h):
    "anorm" (AnormAggregates: a row per record, containment window, top lists are stubs),
    "cassandra" (CassandraAggregates: day-keyed rows clobbered per store, every row returned and
    Monoid-summed, per-service top lists) or "hbase" (HBaseAggregates: reverse-ms row keys, the
    reversed [start, end) scan, Monoid-summed).

    `clock` supplies Time.now in us (tests pin it)."""

    def __init__(self, mode: str = "anorm", services: Optional[Dictionary] = None,
                 annotations: Optional[Dictionary] = None, clock=now_us):
        self._L = _abi.lib()
        m = {"anorm": _abi.ZK_STORE_ANORM, "cassandra": _abi.ZK_STORE_CASSANDRA, "hbase": _abi.ZK_STORE_HBASE}[mode]
        h = C.c_void_p()
        st = self._L.zk_store_create(m, C.byref(h))
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, _abi.status_str(st))
        self._h = h
        self.mode = mode
        self.services = services if services is not None else Dictionary()
        self.annotations = annotations if annotations is not None else Dictionary()
        self.clock = clock

    def _check(self, st: int) -> None:
        if st != _abi.ZK_OK:
            raise _abi.ZkError(st, self._L.zk_store_last_error(self._h).decode() or _abi.status_str(st))

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.zk_store_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- dependencies -------------------------------------------------------------------------
    def storeDependencies(self, dependencies: Dependencies) -> None:
        links = dependencies.links
        n = len(links)
        if isinstance(links, LinkList):  # a job's compact record: remap its ids to this store's names
            raw, names = links.compact()
            remap = np.array([self.services.id(x) for x in names] or [0], np.uint32)
            if np.array_equal(remap, np.arange(len(remap), dtype=np.uint32)):
                arr = raw  # the same ids (a store fed by one job): no remapped copy
            else:
                arr = raw.copy()
                arr["parent"] = remap[raw["parent"]]
                arr["child"] = remap[raw["child"]]
            self._check(self._L.zk_store_put_dependencies(self._h, int(dependencies.start_time),
                                                          int(dependencies.end_time), arr.ctypes.data, n))
            return
        arr = (_abi.zk_dep_link * max(n, 1))()
        for i, l in enumerate(links):
            arr[i] = _abi.zk_dep_link(self.services.id(l.parent.name), self.services.id(l.child.name),
                                      _to_c(l.duration_moments))
        self._check(self._L.zk_store_put_dependencies(self._h, int(dependencies.start_time),
                                                      int(dependencies.end_time), arr, n))

    def getDependencies(self, startDate: Optional[int], endDate: Optional[int] = None) -> Dependencies:
        s = C.c_int64(startDate) if startDate is not None else None
        e = C.c_int64(endDate) if endDate is not None else None
        now = int(self.clock())
        n = C.c_uint64()
        rs, re_ = C.c_int64(), C.c_int64()
        sp = C.byref(s) if s is not None else None
        ep = C.byref(e) if e is not None else None
        self._check(self._L.zk_store_get_dependencies(self._h, sp, ep, now, None, 0, C.byref(n), None, None))
        arr = (_abi.zk_dep_link * max(n.value, 1))()
        self._check(self._L.zk_store_get_dependencies(self._h, sp, ep, now, arr, n.value, C.byref(n),
                                                      C.byref(rs), C.byref(re_)))
        links = tuple(
            DependencyLink(Service(self.services.name(arr[i].parent)), Service(self.services.name(arr[i].child)),
                           _from_c(arr[i].moments))
            for i in range(n.value)
        )
        return Dependencies(int(rs.value), int(re_.value), links)

    def count(self) -> int:
        n = C.c_uint64()
        self._check(self._L.zk_store_count(self._h, C.byref(n)))
        return int(n.value)

    def watermark(self) -> int:
        """IFNULL(MAX(end_ts), 0) over every stored row (AnormAggregator.scala:62-66)."""
        w = C.c_int64()
        self._check(self._L.zk_store_watermark(self._h, C.byref(w)))
        return int(w.value)

    # -- top annotations ----------------------------------------------------------------------
    def _put_top(self, kind: int, serviceName: str, a: Sequence[str]) -> None:
        ids = np.array([self.annotations.id(x) for x in a], dtype=np.uint64)
        self._check(self._L.zk_store_put_top(self._h, kind, self.services.id(serviceName),
                                             ids.ctypes.data if len(ids) else None, len(ids)))

    def _get_top(self, kind: int, serviceName: str) -> List[str]:
        svc = self.services.get(serviceName)
        if svc is None:
            return []
        n = C.c_uint64()
        self._check(self._L.zk_store_get_top(self._h, kind, svc, None, 0, C.byref(n)))
        ids = np.zeros(max(n.value, 1), np.uint64)
        self._check(self._L.zk_store_get_top(self._h, kind, svc, ids.ctypes.data, n.value, C.byref(n)))
        return [self.annotations.name(int(i)) for i in ids[: n.value]]

    def storeTopAnnotations(self, serviceName: str, a: Sequence[str]) -> None:
        self._put_top(_abi.ZK_TOP_ANNOTATIONS, serviceName, a)

    def storeTopKeyValueAnnotations(self, serviceName: str, a: Sequence[str]) -> None:
        self._put_top(_abi.ZK_TOP_KV_ANNOTATIONS, serviceName, a)

    def getTopAnnotations(self, serviceName: str) -> List[str]:
        return self._get_top(_abi.ZK_TOP_ANNOTATIONS, serviceName)

    def getTopKeyValueAnnotations(self, serviceName: str) -> List[str]:
        return self._get_top(_abi.ZK_TOP_KV_ANNOTATIONS, serviceName)


def dependencies_to_thrift(deps: Dependencies) -> bytes:
    """The record as the Cassandra store keeps it: TBinaryProtocol thriftscala.Dependencies
    (zipkinDependencies.thrift:24-43 via WrappedDependencies.toThrift, thrift.scala:330-333)."""
    names = Dictionary()
    arr = (_abi.zk_dep_link * max(1, len(deps.links)))()
    for i, l in enumerate(deps.links):
        arr[i].parent = names.id(l.parent.name)
        arr[i].child = names.id(l.child.name)
        arr[i].moments = _to_c(l.duration_moments)
    raw = [names.name(i).encode() for i in range(len(names))]
    ptrs = (C.c_char_p * max(1, len(raw)))(*raw)
    lens = (C.c_uint32 * max(1, len(raw)))(*[len(b) for b in raw])
    L = _abi.lib()
    n = C.c_uint64()
    args = (int(deps.start_time), int(deps.end_time), arr, len(deps.links), ptrs, lens, len(raw))
    st = L.zk_dependencies_encode(*args, None, 0, C.byref(n))
    if st != _abi.ZK_OK:
        raise _abi.ZkError(st, _abi.status_str(st))
    buf = (C.c_uint8 * max(1, n.value))()
    st = L.zk_dependencies_encode(*args, buf, n.value, C.byref(n))
    if st != _abi.ZK_OK:
        raise _abi.ZkError(st, _abi.status_str(st))
    return bytes(buf)[: n.value]


def dependencies_from_thrift(data: bytes) -> Dependencies:
    """ThriftDependencies.toDependencies (thrift.scala:335-340) of a stored column value."""
    from .ingest import SpanDecoder

    dec = SpanDecoder()  # its dictionary maps the stored names to link ids
    L = _abi.lib()
    src = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    start, end, n = C.c_int64(), C.c_int64(), C.c_uint64()
    dec._check(L.zk_dependencies_decode(dec._h, src, len(data), C.byref(start), C.byref(end), None, 0, C.byref(n)))
    arr = (_abi.zk_dep_link * max(1, n.value))()
    dec._check(L.zk_dependencies_decode(dec._h, src, len(data), C.byref(start), C.byref(end), arr, n.value,
                                        C.byref(n)))
    links = tuple(DependencyLink(Service(dec.service_name(arr[i].parent)), Service(dec.service_name(arr[i].child)),
                                 _from_c(arr[i].moments)) for i in range(n.value))
    return Dependencies(start.value, end.value, links)


def cassandra_row_key(start_time_us: int) -> int:
    """CassandraAggregates.storeDependencies row key: startTime.floor(1.day) in us."""
    return int(_abi.lib().zk_dependencies_row_key(int(start_time_us)))


def links_from_table(table, services: Dictionary) -> "LinkList":
    """The present cells of a finalized host LinkTable as DependencyLinks (zk_link_table_compact),
    kept in the table's form (LinkList) until read."""
    return LinkList(table, [services.name(i) for i in range(min(table.num_services, len(services)))])


class ZipkinAggregateJob:
    """ZipkinAggregateJob.scala:10-46 with the compute on the device.

    run(batches) accumulates column batches (one record per stored span fragment, service ids from
    `services`; host SpanColumns or device DeviceColumns), finalizes, and returns
    Dependencies(Time(0), Time.now, links) -- or None when there is no link, in which case the
    reference writes nothing (:43-45). With an `aggregates` sink the record is stored through
    storeDependencies (StorageRecordWriter.scala:13-17).

    order="any" (default): each batch holds whole traces, its fragments in any order -- what the
    reference's groupBy traceId accepts (:21-22, 28-33); the device clusters every batch. With
    verify=True (the default) a trace that recurs in a later batch fails the job
    (ZK_ERR_NOT_CLUSTERED) instead of being joined in two halves.
    order="rows": batches as a row-per-trace storage reader returns them
    (StorageRecordReader.scala:49-54) -- every trace's fragments adjacent, a trace possibly cut at a
    batch edge -- accumulated with ZK_BATCH_TRACE_CLUSTERED | ZK_BATCH_CONTINUES, the path bench.py
    measures. A caller opts in to it for input it knows to be row-ordered; verify=True then also
    checks that promise exactly on the device (a split trace fails the job), verify=False trusts it.

    The device context is kept between runs (a scheduled job reuses its buffers); close() frees it.
    """

    def __init__(self, services: Dictionary, *, device: int = 0, strict: bool = True,
                 aggregates: Optional[Aggregates] = None, clock=now_us, order: str = "any", verify: bool = True):
        if order not in ("rows", "any"):
            raise ValueError("order is 'rows' or 'any'")
        self.services = services
        self.device = device
        self.strict = strict
        self.aggregates = aggregates
        self.clock = clock
        self.order = order
        self.verify = verify
        self.stats: dict = {}
        self._ctx = None

    def close(self) -> None:
        if self._ctx is not None:
            self._ctx.close()
            self._ctx = None

    def _context(self, S: int):
        from .context import DepsContext

        if self._ctx is None or self._ctx.num_services != S:
            self.close()
            self._ctx = DepsContext(S, device=self.device, strict=self.strict)
        else:
            self._ctx.reset()
        return self._ctx

    def accumulate_all(self, batches, num_services: Optional[int] = None):
        """The job up to the finalize: every batch into a reset context (returned)."""
        from .columns import SpanColumns

        if isinstance(batches, SpanColumns) or hasattr(batches, "abi"):
            batches = [batches]
        ctx = self._context(num_services or max(1, len(self.services)))
        rows = self.order == "rows"
        for b in batches:
            ctx.accumulate(b, clustered=rows, continues=rows, verify=self.verify)
        return ctx

    def run(self, batches, num_services: Optional[int] = None) -> Optional[Dependencies]:
        ctx = self.accumulate_all(batches, num_services)
        table = ctx.finalize()  # the job ends here: a held-back trace is aggregated first
        self.stats = ctx.stats()
        return self._publish(table)

    def _publish(self, table) -> Optional[Dependencies]:
        links = links_from_table(table, self.services)
        if not links:
            return None
        deps = Dependencies(0, int(self.clock()), links)  # Time.fromMilliseconds(0), Time.now (:41-42)
        if self.aggregates is not None:
            self.aggregates.storeDependencies(deps)
        return deps


def publish_top_kv(sketch, aggregates: GpuAggregates, keys: Dict[int, str], k: int = 10) -> None:
    """The removed producer of storeTopKeyValueAnnotations (CHANGELOG:7-8): the device count-min
    top-K of every service, key hashes mapped back to key strings by `keys` ({hash: key}), stored
    per service as the reference's per-service list (CassandraAggregates.scala:100-102)."""
    kk, est, cnt = sketch.topk_all(k)
    for s in range(sketch.num_services):
        if cnt[s] == 0 or s >= len(aggregates.services):
            continue
        names = [keys[int(h)] for h in kk[s][: cnt[s]]]
        aggregates.storeTopKeyValueAnnotations(aggregates.services.name(s), names)


class StoredSpanJob:
    """The aggregation job fed from the stored span bytes, with the removed producers of the
    top-annotation lists (CHANGELOG:7-8) restored next to it.

    Input: batches of stored fragments (the Cassandra column values, i.e.
    Snappy(TBinaryProtocol(Span)), CassieSpanStore.scala:52; a list of bytes or the packed
    (buf, offsets) form of SpanDecoder.decode) in row order: a row-per-trace reader
    (StorageRecordReader.scala:49-54) returns every trace's fragments together and may cut a trace at
    a batch edge. run() streams them: a worker thread decodes batch k+1 on the host (include/
    zkingest.h: the 48-B records plus the span indexer's items, CassieSpanStore.scala:214-242) while
    batch k runs on the device -- the dependency job (ZipkinAggregateJob.scala:20-43, accumulated with
    ZK_BATCH_TRACE_CLUSTERED | ZK_BATCH_CONTINUES) and one count-min + top-K sketch each for
    binary-annotation keys and non-core annotation values. run_device() takes fragments already in
    HBM through the device decoder, which emits the same indexer items on the device
    (zk_ingest_dev_spans_items; indexer=False: dependencies only, the decoder's faster build).
    Output, through `aggregates`: storeDependencies, storeTopKeyValueAnnotations and
    storeTopAnnotations per service (Aggregates.scala:31-36).

    max_services sizes the device table (S x S cells) and the sketches before the dictionary is
    known; a stream that names more services fails with ZK_ERR_SERVICE_RANGE. For the same reason the
    count-min width per service is kv_width or the largest, 4096 (the auto width of <= 256 services).
    """

    def __init__(self, *, device: int = 0, strict: bool = True, aggregates: Optional[Aggregates] = None,
                 clock=now_us, top_k: int = 10, snappy: bool = True, kv_width: int = 0, seed: int = 0,
                 max_services: int = 1024, verify: bool = False):
        self.device = device
        self.strict = strict
        self.aggregates = aggregates
        self.clock = clock
        self.top_k = top_k
        self.snappy = snappy
        self.kv_width = kv_width
        self.seed = seed
        self.max_services = max_services
        self.verify = verify
        self.stats: dict = {}
        self.rejected = 0
        self.services: Optional[Dictionary] = None
        self.top_kv: Dict[str, List[str]] = {}
        self.top_annotations: Dict[str, List[str]] = {}

    def _decode(self, dec, blobs):
        n = len(blobs[1]) - 1 if isinstance(blobs, tuple) else len(blobs)
        cap = max(16, 8 * n)
        while True:
            try:
                return dec.decode(blobs, snappy=self.snappy, strict=self.strict, items=True, item_cap=cap), n
            except _abi.ZkError as e:
                if e.status != _abi.ZK_ERR_CAPACITY:
                    raise
                cap *= 4  # more binary annotations than guessed: decode the batch again

    def _tops(self, dec, sketch, S) -> Dict[str, List[str]]:
        keys, _, cnt = sketch.topk_all(self.top_k)
        kl, cl = keys[:S].tolist(), cnt[:S].tolist()  # Python ints: no numpy scalar per lookup
        return {dec.service_name(s_): [dec.string(h) for h in kl[s_][: cl[s_]]] for s_ in range(S) if cl[s_]}

    def _finish(self, ctx, names: List[str]) -> Optional[Dependencies]:
        if len(names) > self.max_services:
            raise _abi.ZkError(_abi.ZK_ERR_SERVICE_RANGE, f"{len(names)} services > max_services {self.max_services}")
        self.services = Dictionary(names)
        table = ctx.finalize()
        self.stats = ctx.stats()
        job = ZipkinAggregateJob(self.services, device=self.device, strict=self.strict, clock=self.clock)
        return job._publish(table)

    def run(self, batches) -> Optional[Dependencies]:
        from concurrent.futures import ThreadPoolExecutor

        from .context import DepsContext
        from .ingest import SpanDecoder
        from .kv import KvSketch

        dec = SpanDecoder()
        self.rejected = 0
        S = self.max_services
        with DepsContext(S, device=self.device, strict=self.strict) as ctx, \
                KvSketch(S, device=self.device, width=self.kv_width or 4096, seed=self.seed) as kvs, \
                KvSketch(S, device=self.device, width=self.kv_width or 4096, seed=self.seed) as anns, \
                ThreadPoolExecutor(max_workers=1) as pool:
            it = iter(batches)
            nxt = next(it, None)
            fut = pool.submit(self._decode, dec, nxt) if nxt is not None else None
            cap = self.device_accumulate_records
            pend, gn = [], 0  # the items of a group of batches (run_device's decode groups)

            def items_in():
                nonlocal pend, gn
                for k, sk in ((0, kvs), (2, anns)):
                    svc = np.concatenate([p[k] for p in pend]) if pend else np.zeros(0, np.uint32)
                    if len(svc):
                        sk.accumulate(svc, np.concatenate([p[k + 1] for p in pend]))
                pend, gn = [], 0

            while fut is not None:
                (cols, rej, (ks, kh), (as_, ah)), n = fut.result()  # n: the batch's fragments
                nxt = next(it, None)
                # the decoder's C call releases the GIL: batch k+1 decodes while batch k is staged and runs
                fut = pool.submit(self._decode, dec, nxt) if nxt is not None else None
                self.rejected += rej
                ctx.accumulate(cols, clustered=True, continues=True, verify=self.verify)
                # the sketches take consecutive batches of up to `cap` fragments together, as
                # run_device's decode groups do, so both drivers store the same top lists
                if gn + n > cap or n > cap:
                    items_in()
                pend.append((ks, kh, as_, ah))
                gn += n
                if n > cap:
                    items_in()
            items_in()
            names = dec.service_names()
            deps = self._finish(ctx, names)
            self.top_kv = self._tops(dec, kvs, len(names))
            self.top_annotations = self._tops(dec, anns, len(names))
        if self.aggregates is not None:
            if deps is not None:
                self.aggregates.storeDependencies(deps)
            for name, keys in self.top_kv.items():
                self.aggregates.storeTopKeyValueAnnotations(name, keys)
            for name, values in self.top_annotations.items():
                self.aggregates.storeTopAnnotations(name, values)
        return deps

    # run_device: consecutive batches are decoded together (one zk_ingest_dev_spans_multi call per
    # group of up to this many fragments) into one column buffer and accumulated together
    # (row-order batches back to back are one row-order batch, and the dependency sums do not depend
    # on where batches are cut), so a stream of small batches pays the decoder's and the
    # accumulate's fixed costs once per buffer instead of once per batch
    device_accumulate_records = 1 << 24

    def _device_state(self, indexer: bool):
        """The device objects of run_device, kept between runs (a scheduled job reuses its buffers,
        as ZipkinAggregateJob keeps its context): stream, decoder (its service dictionary and string
        map persist: ids stay stable, outputs are by name), context, gathering buffer and the two
        sketches, reset at the start of every run. close() frees them. The dictionary persisting,
        max_services bounds the distinct services over the job's lifetime, not per run."""
        import torch

        from .context import DepsContext
        from .ingest import DeviceSpanDecoder
        from .kv import KvSketch

        st = getattr(self, "_dev", None)
        if st is None:
            S = self.max_services
            stream = torch.cuda.Stream(device=self.device)
            st = {"stream": stream, "pool": None,
                  "dec": DeviceSpanDecoder(max(4096, S), device=self.device, stream=stream.cuda_stream),
                  "ctx": DepsContext(S, device=self.device, strict=self.strict, stream=stream.cuda_stream),
                  "kvs": None, "anns": None}
            self._dev = st
        else:
            st["ctx"].reset()
        if indexer:
            for k in ("kvs", "anns"):
                if st[k] is None:
                    st[k] = KvSketch(self.max_services, device=self.device, stream=st["stream"].cuda_stream,
                                     width=self.kv_width or 4096, seed=self.seed)
                else:
                    st[k].reset()
        return st

    def close(self) -> None:
        st = getattr(self, "_dev", None)
        if st is not None:
            for k in ("kvs", "anns", "ctx", "dec"):
                if st[k] is not None:
                    st[k].close()
            self._dev = None

    def run_device(self, batches, *, indexer: bool = True) -> Optional[Dependencies]:
        """batches: (buf uint8, offsets int64[n + 1], n) torch tensors already in HBM, in row order.
        Decoded on the device into a reused column buffer and accumulated on the same stream, several
        small batches at a time (device_accumulate_records); with `indexer` the decoder's items feed
        the two count-min + top-K sketches batch by batch as in run(). The device objects are kept
        for the next run (close() frees them)."""
        import torch

        from .columns import DeviceColumns

        self.rejected = 0
        t0 = time.perf_counter()
        st = self._device_state(indexer)
        stream, dec, ctx, kvs, anns = st["stream"], st["dec"], st["ctx"], st["kvs"], st["anns"]
        t1 = time.perf_counter()
        cap = self.device_accumulate_records
        filled = 0
        cols = None  # a batch larger than the gathering buffer: its own columns
        group, gn = [], 0  # consecutive batches decoded together (one decode call)

        def flush():
            nonlocal filled
            if filled:
                ctx.accumulate(st["pool"].slice(0, filled), clustered=True, continues=True, verify=self.verify)
                filled = 0

        def items_in(ks, kh, as_, ah):
            if len(ks):
                kvs.accumulate(ks, kh)
            if len(as_):
                anns.accumulate(as_, ah)

        def decode_group():
            # the group's batches joined in one decode (zk_ingest_dev_spans_multi) straight into the
            # gathering buffer: one set of launches and one host round trip for all of them
            nonlocal filled, group, gn
            if not group:
                return
            pool = st["pool"]
            if pool is None or filled + gn > pool.capacity:
                flush()
                if pool is None or gn > pool.capacity:  # grown on demand, up to `cap` records
                    pool = st["pool"] = None
                    pool = st["pool"] = DeviceColumns(min(cap, max(gn, 1 << 20)), device=f"cuda:{self.device}")
            out = pool.slice(filled, filled + gn)
            # the caller's tensors may still be in flight on its current stream (a non_blocking copy,
            # a kernel that writes them; a lazy iterator makes each batch just before it is read):
            # the job's stream waits for everything queued there
            stream.wait_stream(torch.cuda.current_stream(self.device))
            if indexer:
                out, rej, (ks, kh), (as_, ah) = dec.decode_device_many(
                    group, snappy=self.snappy, strict=self.strict, out=out, items=True)
                items_in(ks, kh, as_, ah)
            else:
                out, rej = dec.decode_device_many(group, snappy=self.snappy, strict=self.strict, out=out)
            self.rejected += rej
            filled += out.n
            group, gn = [], 0

        try:
            for buf, off, n in batches:
                # the caller's allocator keeps the batch's memory until the job's stream is done
                buf.record_stream(stream)
                off.record_stream(stream)
                if n <= cap:
                    if gn + n > cap:
                        decode_group()
                    group.append((buf, off, n))
                    gn += n
                    continue
                decode_group()
                flush()
                stream.wait_stream(torch.cuda.current_stream(self.device))
                if cols is None or cols.capacity < n:
                    cols = None
                if indexer:
                    cols, rej, (ks, kh), (as_, ah) = dec.decode_device(
                        buf, off, n, snappy=self.snappy, strict=self.strict, out=cols, items=True)
                    items_in(ks, kh, as_, ah)
                else:
                    cols, rej = dec.decode_device(buf, off, n, snappy=self.snappy, strict=self.strict, out=cols)
                self.rejected += rej
                ctx.accumulate(cols, clustered=True, continues=True, verify=self.verify)
            decode_group()
            flush()
            t2 = time.perf_counter()
            names = dec.service_names()
            deps = self._finish(ctx, names)
            if indexer:
                self.top_kv = self._tops(dec, kvs, len(names))
                self.top_annotations = self._tops(dec, anns, len(names))
            t3 = time.perf_counter()
        except BaseException:
            self.close()  # a failed run leaves no half-used state behind
            raise
        if self.aggregates is not None:
            if deps is not None:
                self.aggregates.storeDependencies(deps)
            if indexer:
                for name, keys in self.top_kv.items():
                    self.aggregates.storeTopKeyValueAnnotations(name, keys)
                for name, values in self.top_annotations.items():
                    self.aggregates.storeTopAnnotations(name, values)
        # where the run's wall time went (ms): device objects ready, the batches decoded and
        # accumulated, finalize + the record (+ the top lists), the store calls
        self.phase_ms = {"setup": (t1 - t0) * 1e3, "batches": (t2 - t1) * 1e3, "finish": (t3 - t2) * 1e3,
                         "store": (time.perf_counter() - t3) * 1e3}
        return deps
