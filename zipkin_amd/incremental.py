"""Watermark-incremental dependency runs.

The reference's incremental driver is AnormAggregator
(zipkin-anormdb/.../aggregates/AnormAggregator.scala:32-121). Its driver logic:

* the watermark is the latest end time of the stored dependencies, 0 when there are none
  (`SELECT IFNULL(MAX(END_TS), 0) FROM zipkin_dependencies`, :62-66);
* only spans created after the watermark are aggregated (:64, :77-80); with none, nothing is
  stored ("already up-to-date", :52-55);
* the new spans are cut into max(spanCount / 10000, 1) time steps over [minTime, maxTime]
  (SpanSummary, :35-39), each step's links become Dependencies(stepStart, stepEnd, links) and the
  steps are Monoid-summed (:95-113) into ONE stored record (:43-56).

Its SQL join is not the job's (no traceId, one row per annotation: SURVEY.md §8a A15), so this
driver keeps that driver logic and runs the real job (ZipkinAggregateJob.scala:20-43, on the
device) over the new part:

* the unit is the trace, because the job needs trace-complete batches: a trace is new when its
  created time -- the latest `created_ts` of its fragments -- is after the watermark, and then
  all of its fragments are aggregated;
* the record's time range follows the reference's steps: with min/max the earliest/latest created
  time of the new traces and `count` their records, steps = max(count / 10000, 1) and
  stepSize = (max - min) / steps (SpanSummary, :35-39); the steps run over
  Range.Long(min, max + 1, stepSize), so the record is Dependencies(min, last boundary, links)
  (:43-49, :102-120) and the traces created after the last boundary wait for the next run, as
  the reference's spans do. The first step is the half-open (min, boundary] of the reference's
  `created_ts > start` with start = min (:46-47, :79), so the traces created exactly at min are
  skipped for good, as the reference skips those spans. (All new traces created at one instant
  make stepSize 0, where the reference's Range throws; here they are aggregated and the record
  ends at that instant.)
* the record is stored whenever new traces exist, with or without links: the reference folds
  from Monoid.zero and always stores the result (:41-56), which is what advances the watermark;
* one device job over the selected traces replaces the per-step Monoid sum; the two differ only
  in the rounding of m1..m4 (the device's are exactly rounded; m0 is identical).

The next run's watermark is that record's end, so a trace is aggregated exactly once as long as
traces are complete when their created time passes the watermark (the reference assumes the same
of spans).
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from .aggregates import Dependencies, GpuAggregates, ZipkinAggregateJob
from .columns import SpanColumns


def trace_created(cols: SpanColumns, created_ts) -> np.ndarray:
    """The created time of each record's trace: the latest created_ts among the trace's
    fragments. Batches are trace-clustered: a trace is a maximal run of equal trace_id."""
    created = np.asarray(created_ts, dtype=np.int64)
    n = len(cols)
    if created.shape != (n,):
        raise ValueError(f"created_ts must hold one time per record ({n})")
    if n == 0:
        return np.zeros(0, np.int64)
    tid = cols.trace_id
    start = np.ones(n, bool)
    start[1:] = tid[1:] != tid[:-1]
    per_trace = np.maximum.reduceat(created, np.flatnonzero(start))
    return per_trace[np.cumsum(start) - 1]


class IncrementalAggregator:
    """AnormAggregator.apply() (AnormAggregator.scala:41-57) over the device job.

    `aggregates` is the store the watermark is read from and the record is written to; its
    `services` dictionary names the batch's service ids. `job` defaults to the device
    ZipkinAggregateJob (anything with the same run(batch, num_services) works)."""

    def __init__(self, aggregates: GpuAggregates, *, device: int = 0, strict: bool = True, job=None):
        self.aggregates = aggregates
        self.job = job if job is not None else ZipkinAggregateJob(aggregates.services, device=device,
                                                                   strict=strict)
        self.last_selected = 0  # records aggregated by the last apply()

    def watermark(self) -> int:
        """IFNULL(MAX(END_TS), 0) over every stored row (AnormAggregator.scala:64)."""
        return self.aggregates.watermark()

    def apply(self, cols: SpanColumns, created_ts, num_services: Optional[int] = None) -> Optional[Dependencies]:
        """Aggregate the traces created after the watermark, up to the last step boundary, and
        store their Dependencies; returns the stored record, or None when nothing is new."""
        wm = self.watermark()
        created = trace_created(cols, created_ts)
        new = created > wm
        count = int(new.sum())
        if not count:
            self.last_selected = 0
            return None  # "Aggregated span dependencies already up-to-date" (:52-55)
        lo, hi = int(created[new].min()), int(created[new].max())
        steps = max(count // 10000, 1)
        step = (hi - lo) // steps
        end = hi if step == 0 else lo + ((hi - lo) // step) * step
        # the reference's first step queries created_ts > minTime with start = minTime
        # (AnormAggregator.scala:46-47,79): spans created exactly at minTime are never aggregated,
        # and the stored record's end moves the watermark past them. (stepSize 0 -- every new trace
        # created at one instant -- makes the reference's Range throw; here those traces are kept.)
        sel = new & (created <= end)
        if step != 0:
            sel &= created > lo
        self.last_selected = int(sel.sum())
        deps = self.job.run(cols.take(np.flatnonzero(sel)), num_services=num_services)
        rec = Dependencies(lo, end, deps.links if deps is not None else ())
        self.aggregates.storeDependencies(rec)
        return rec
