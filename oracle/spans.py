"""TEST INFRASTRUCTURE ONLY — span-level restatement of the reference semantics.

Pure Python, for small inputs. Every function cites the reference file:line it restates
(paths relative to /root/reference, `.../` = src/main/scala/com/twitter/zipkin/):

* Endpoint / Annotation / BinaryAnnotation / Span:  zipkin-common/.../common/*.scala
* thrift ingest validation:  zipkin-scrooge/.../conversions/thrift.scala:36-45,64-75,99-121
* the job:  zipkin-aggregate/.../aggregate/ZipkinAggregateJob.scala:20-43
* Dependencies monoid:  zipkin-common/.../common/Dependencies.scala:36-83

The reference leaves the reduce order of `mergeSpan` unspecified; this oracle reduces fragments in
input order (a left fold), which is one of the orders the reference may pick.
"""
from __future__ import annotations

from collections import OrderedDict, defaultdict
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

from .moments import ZERO, Moments, algebird_fold, algebird_plus, exact_moments

# zipkin-common/.../Constants.scala:20-32
CLIENT_SEND, CLIENT_RECV, SERVER_SEND, SERVER_RECV = "cs", "cr", "ss", "sr"
CORE_CLIENT = (CLIENT_SEND, CLIENT_RECV)
CORE_SERVER = (SERVER_RECV, SERVER_SEND)
CORE_ANNOTATIONS = (CLIENT_SEND, CLIENT_RECV, SERVER_RECV, SERVER_SEND)
UNKNOWN_SERVICE_NAME = "Unknown service name"  # Endpoint.UnknownServiceName


class NoServiceNameError(Exception):
    """The reference's `parent.serviceName.get` on None (ZipkinAggregateJob.scala:36-37)."""


class IncompleteTraceDataError(Exception):
    pass


@dataclass(frozen=True)
class Endpoint:
    ipv4: int
    port: int
    service_name: str


@dataclass(frozen=True)
class Annotation:
    timestamp: int
    value: str
    host: Optional[Endpoint] = None
    duration: Optional[int] = None


@dataclass(frozen=True)
class BinaryAnnotation:
    key: str
    value: bytes
    annotation_type: str = "String"
    host: Optional[Endpoint] = None


@dataclass(frozen=True)
class Span:
    trace_id: int
    name: str
    id: int
    parent_id: Optional[int]
    annotations: Tuple[Annotation, ...] = ()
    binary_annotations: Tuple[BinaryAnnotation, ...] = ()
    debug: bool = False

    # Span.scala:119-120
    @property
    def service_names(self) -> set:
        return {a.host.service_name.lower() for a in self.annotations if a.host is not None}

    # Span.scala:216-223
    def client_side_annotations(self) -> List[Annotation]:
        return [a for a in self.annotations if a.value in CORE_CLIENT]

    def server_side_annotations(self) -> List[Annotation]:
        return [a for a in self.annotations if a.value in CORE_SERVER]

    # Span.scala:125-131
    @property
    def service_name(self) -> Optional[str]:
        if not self.annotations:
            return None
        for a in self.server_side_annotations():
            if a.host is not None:
                return a.host.service_name
        for a in self.client_side_annotations():
            if a.host is not None:
                return a.host.service_name
        return None

    # Span.scala:148-169
    def merge_span(self, other: "Span") -> "Span":
        if self.id != other.id:
            raise ValueError("Span ids must match")
        name = other.name if self.name in ("", "Unknown") else self.name
        return Span(
            self.trace_id,
            name,
            self.id,
            self.parent_id,
            self.annotations + other.annotations,
            self.binary_annotations + other.binary_annotations,
            self.debug or other.debug,
        )

    # Span.scala:174-191 with Span.timestampOrdering (:72-74); Scala's List.min/max keep the
    # first of equal elements
    @property
    def first_annotation(self) -> Optional[Annotation]:
        best = None
        for a in self.annotations:
            if best is None or a.timestamp < best.timestamp:
                best = a
        return best

    @property
    def last_annotation(self) -> Optional[Annotation]:
        best = None
        for a in self.annotations:
            if best is None or a.timestamp > best.timestamp:
                best = a
        return best

    # Span.scala:228-230
    @property
    def duration(self) -> Optional[int]:
        f, l = self.first_annotation, self.last_annotation
        if f is None or l is None:
            return None
        return l.timestamp - f.timestamp

    # Span.scala:236-240
    @property
    def is_valid(self) -> bool:
        return all(sum(1 for a in self.annotations if a.value == c) <= 1 for c in CORE_ANNOTATIONS)

    # Span.scala:208-211
    def is_client_side(self) -> bool:
        return any(a.value in (CLIENT_SEND, CLIENT_RECV) for a in self.annotations)

    def get_annotation(self, value: str) -> Optional[Annotation]:
        return next((a for a in self.annotations if a.value == value), None)

    def get_binary_annotation(self, key: str) -> Optional[BinaryAnnotation]:
        return next((b for b in self.binary_annotations if b.key == key), None)

    def annotations_as_map(self) -> Dict[str, Annotation]:
        return {a.value: a for a in self.annotations}


# ---- thrift ingest validation (thrift.scala) ------------------------------------------------
def thrift_endpoint(ipv4: int, port: int, service_name: Optional[str]) -> Endpoint:
    """thrift.scala:36-43: null/"" service name -> "Unknown service name"."""
    return Endpoint(ipv4, port, UNKNOWN_SERVICE_NAME if service_name in (None, "") else service_name)


def thrift_annotation(timestamp: int, value: str, host: Optional[Endpoint] = None) -> Annotation:
    """thrift.scala:64-73: timestamp <= 0 or "" value are rejected."""
    if timestamp <= 0:
        raise ValueError(f"Annotation must have a timestamp: {timestamp}")
    if value == "":
        raise ValueError("Annotation must have a value")
    return Annotation(timestamp, value, host)


def thrift_span(trace_id, name, id, parent_id, annotations=None, binary_annotations=None, debug=False) -> Span:
    """thrift.scala:99-121: null name throws; null annotation lists become empty."""
    if name is None:
        raise IncompleteTraceDataError("No name set in Span")
    return Span(trace_id, name, id, parent_id, tuple(annotations or ()), tuple(binary_annotations or ()), debug)


# ---- the job ----------------------------------------------------------------------------------
@dataclass
class JobResult:
    durations: Dict[Tuple[str, str], List[int]]  # (parent svc, child svc) -> child durations
    merged: Dict[Tuple[int, int], Span]
    no_service: int = 0

    def exact(self) -> Dict[Tuple[str, str], Moments]:
        return {k: exact_moments(v) for k, v in self.durations.items()}

    def algebird(self) -> Dict[Tuple[str, str], Moments]:
        return {k: algebird_fold(float(d) for d in v) for k, v in self.durations.items()}


def aggregate_job(spans: Iterable[Span], strict: bool = True) -> JobResult:
    """ZipkinAggregateJob.scala:20-43 on in-memory spans."""
    groups: "OrderedDict[Tuple[int, int], Span]" = OrderedDict()
    for s in spans:  # :21-22 groupBy((id, traceId)).reduce(mergeSpan) — left fold in input order
        k = (s.id, s.trace_id)
        groups[k] = groups[k].merge_span(s) if k in groups else s
    valid = OrderedDict((k, s) for k, s in groups.items() if s.is_valid)  # :23
    durations: Dict[Tuple[str, str], List[int]] = defaultdict(list)
    no_service = 0
    for k, child in valid.items():  # :28-31 children keyed by (parentId, traceId)
        if child.parent_id is None:
            continue
        parent = valid.get((child.parent_id, child.trace_id))  # :33 inner join
        if parent is None:
            continue
        ps, cs = parent.service_name, child.service_name  # :36-37 serviceName.get
        if ps is None or cs is None:
            if strict:
                raise NoServiceNameError(f"span {child.id} in trace {child.trace_id}")
            no_service += 1
            continue
        d = child.duration  # :35 Moments(d) | Monoid.zero (unreachable once the name exists)
        durations[(ps, cs)].append(d)
    return JobResult(dict(durations), dict(groups), no_service)


# ---- Dependencies monoid (Dependencies.scala) ------------------------------------------------
@dataclass(frozen=True)
class DependencyLink:
    parent: str
    child: str
    moments: Moments

    def plus(self, other: "DependencyLink") -> "DependencyLink":  # Dependencies.scala:38-43
        assert self.parent == other.parent and self.child == other.child
        return DependencyLink(self.parent, self.child, algebird_plus(self.moments, other.moments))


TIME_TOP = 2**63 - 1  # Time.Top / Time.Bottom stand-ins for the monoid zero
TIME_BOTTOM = -(2**63)


@dataclass(frozen=True)
class Dependencies:
    start_time: int
    end_time: int
    links: Tuple[DependencyLink, ...] = ()

    @staticmethod
    def zero() -> "Dependencies":  # Dependencies.scala:81
        return Dependencies(TIME_TOP, TIME_BOTTOM, ())

    def plus(self, r: "Dependencies") -> "Dependencies":  # Dependencies.scala:68-79
        start = min(r.start_time, self.start_time)
        end = max(r.end_time, self.end_time)
        lmap = {(l.parent, l.child): l for l in self.links}
        rmap = {(l.parent, l.child): l for l in r.links}
        merged = dict(rmap)
        for k, l in lmap.items():  # Monoid.plus(rLinkMap, lLinkMap): r's value first
            merged[k] = merged[k].plus(l) if k in merged else l
        return Dependencies(start, end, tuple(merged.values()))


def merge_dependency_links(links: Sequence[DependencyLink]) -> List[DependencyLink]:
    """DependencyLink.mergeDependencyLinks (Dependencies.scala:45-50)."""
    by: Dict[Tuple[str, str], List[DependencyLink]] = defaultdict(list)
    for l in links:
        by[(l.parent, l.child)].append(l)
    out = []
    for ls in by.values():
        acc = ls[0]
        for l in ls[1:]:
            acc = acc.plus(l)
        out.append(acc)
    return out


# ---- ingest to the columnar record ---------------------------------------
def span_to_record(span: Span, service_ids: Dict[str, int]) -> dict:
    """One stored fragment -> the 48-byte columnar record of include/zkagg.h."""
    flags = 0
    if span.parent_id is not None:
        flags |= 1
    ts = [a.timestamp for a in span.annotations]
    first = min(ts) if ts else 0
    last = max(ts) if ts else 0
    if ts:
        flags |= 2
    svc = 0
    srv = next((a.host.service_name for a in span.server_side_annotations() if a.host is not None), None)
    cli = next((a.host.service_name for a in span.client_side_annotations() if a.host is not None), None)
    if srv is not None:
        flags |= 8
        svc = service_ids.setdefault(srv, len(service_ids))
    elif cli is not None:
        flags |= 4
        svc = service_ids.setdefault(cli, len(service_ids))
    for shift, c in ((8, CLIENT_SEND), (10, CLIENT_RECV), (12, SERVER_RECV), (14, SERVER_SEND)):
        k = min(2, sum(1 for a in span.annotations if a.value == c))
        flags |= k << shift
    pid = span.parent_id if span.parent_id is not None else 0
    return dict(
        trace_id=span.trace_id & (2**64 - 1),
        span_id=span.id & (2**64 - 1),
        parent_id=pid & (2**64 - 1),
        first_ts=first,
        last_ts=last,
        service_id=svc,
        flags=flags,
    )
