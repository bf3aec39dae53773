"""TEST INFRASTRUCTURE ONLY — Python driver of the C restatement (zk_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module, and only
as the checker. Parity status: see the header of zk_oracle.c and DESIGN.md §Oracle. The span-level
semantics it encodes are pinned by the reference's own unit tests (tests/golden/reference_kats.json,
from SpanTest.scala / DependenciesTest.scala / AnormAggregatesTest.scala); the join/group/sum has no
reference-produced output to pin against (the job has no tests, and no JVM exists here), so that
part is cross-checked against the independent span-level restatement in oracle/spans.py.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import time
from pathlib import Path
from typing import Dict, Tuple

import numpy as np

from .moments import Moments, moments_from_power_sums

HERE = Path(__file__).resolve().parent
LIB = HERE / "_build" / "libzkoracle.so"
CELL_WORDS = 17
STAT_NAMES = (
    "records",
    "merged_spans",
    "valid_spans",
    "invalid_spans",
    "child_spans",
    "joined_links",
    "missing_parent",
    "no_service",
    "ambiguous",
    "spilled_traces",
    "duration_range",
    "service_range",
    "trace_too_large",
)

_lib = None


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = C.CDLL(str(LIB))
        L.zko_aggregate.restype = C.c_int
        L.zko_aggregate.argtypes = [C.c_void_p] * 7 + [C.c_uint64, C.c_uint32, C.c_int, C.c_void_p, C.c_void_p]
        L.zkp_aggregate.restype = C.c_int
        L.zkp_aggregate.argtypes = [C.c_void_p] * 7 + [C.c_uint64, C.c_uint32, C.c_int, C.c_int, C.c_void_p,
                                                       C.c_void_p]
        L.zkv_port.restype = C.c_int
        L.zkv_port.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                               C.c_uint64, C.c_int] + [C.c_void_p] * 6 + [C.POINTER(C.c_double)]
        L.zkr_port.restype = C.c_int
        L.zkr_port.argtypes = [C.c_void_p] * 6 + [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint64, C.c_int,
                                                  C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_double)]
        _lib = L
    return _lib


class OracleResult:
    def __init__(self, S: int, cells: np.ndarray, stats: np.ndarray, seconds: float, threads: int):
        self.S = S
        self.cells = cells.reshape(S * S, CELL_WORDS)
        self.stats = {k: int(stats[i]) for i, k in enumerate(STAT_NAMES)}
        self.seconds = seconds
        self.threads = threads

    def power_sums(self, cell: int) -> Tuple[int, int, int, int, int]:
        row = self.cells[cell]
        vals = [int(row[0])]
        for k in range(4):
            w = row[1 + 4 * k : 5 + 4 * k]
            vals.append(sum(int(w[i]) << (64 * i) for i in range(4)))
        return tuple(vals)  # type: ignore[return-value]

    def present_cells(self) -> np.ndarray:
        return np.flatnonzero(self.cells[:, 0])

    def moments(self) -> Dict[Tuple[int, int], Moments]:
        """Exact Moments per (parent id, child id), rounded once (correctly rounded fp64)."""
        out = {}
        for c in self.present_cells():
            out[(int(c) // self.S, int(c) % self.S)] = moments_from_power_sums(*self.power_sums(int(c)))
        return out

    def dense(self):
        """m0 (uint64) and m1..m4 (float64) dense arrays like the product's finalize."""
        n = self.S * self.S
        m0 = self.cells[:, 0].copy()
        ms = [np.zeros(n) for _ in range(4)]
        for (p, c), m in self.moments().items():
            i = p * self.S + c
            ms[0][i], ms[1][i], ms[2][i], ms[3][i] = m.m1, m.m2, m.m3, m.m4
        return m0, ms


def aggregate(cols, num_services: int, threads: int | None = None) -> OracleResult:
    """Run the restatement on a zipkin_amd.SpanColumns-like object (numpy columns)."""
    return _run(cols, num_services, threads, None)


def aggregate_port(cols, num_services: int, threads: int | None = None, clustered: bool = True) -> OracleResult:
    """The CPU baseline (zk_cpu_port.c): the same job in one pass, trace at a time for clustered
    input or hash-partitioned for any order. Output identical to `aggregate`."""
    return _run(cols, num_services, threads, clustered)


def _run(cols, num_services, threads, port_clustered) -> OracleResult:
    if threads is None:
        threads = min(8, os.cpu_count() or 1)
    L = lib()
    S = num_services
    cells = np.zeros(S * S * CELL_WORDS, np.uint64)
    stats = np.zeros(16, np.uint64)
    arrs = [
        np.ascontiguousarray(cols.trace_id, np.uint64),
        np.ascontiguousarray(cols.span_id, np.uint64),
        np.ascontiguousarray(cols.parent_id, np.uint64),
        np.ascontiguousarray(cols.first_ts, np.int64),
        np.ascontiguousarray(cols.last_ts, np.int64),
        np.ascontiguousarray(cols.service_id, np.uint32),
        np.ascontiguousarray(cols.flags, np.uint32),
    ]
    n = int(arrs[0].shape[0])
    t0 = time.perf_counter()
    if port_clustered is None:
        rc = L.zko_aggregate(*[a.ctypes.data for a in arrs], n, S, threads, cells.ctypes.data, stats.ctypes.data)
    else:
        rc = L.zkp_aggregate(*[a.ctypes.data for a in arrs], n, S, threads, 1 if port_clustered else 0,
                             cells.ctypes.data, stats.ctypes.data)
    dt = time.perf_counter() - t0
    if rc != 0:
        raise MemoryError("oracle allocation failed")
    return OracleResult(S, cells, stats, dt, threads)
