"""Cross-check the columnar C restatement (oracle/zk_oracle.c) against the independent span-level
restatement (oracle/spans.py) on rich TraceGen-shaped spans with injected anomalies."""
import random

import numpy as np
import pytest

from oracle import oracle
from oracle.moments import Moments, algebird_fold, exact_moments, moments_close
from oracle.spans import aggregate_job, span_to_record
from tests.richgen import gen_traces
from zipkin_amd.columns import SpanColumns


def to_columns(spans, service_ids):
    recs = [span_to_record(s, service_ids) for s in spans]
    cols = SpanColumns.empty(len(recs))
    for k in ("trace_id", "span_id", "parent_id", "first_ts", "last_ts", "service_id", "flags"):
        getattr(cols, k)[:] = [r[k] for r in recs]
    return cols


@pytest.mark.parametrize("seed,anomalies,shuffle", [(1, 0.0, False), (2, 0.3, False), (3, 0.3, True)])
def test_c_oracle_equals_span_oracle(seed, anomalies, shuffle):
    spans = gen_traces(seed, 300, max_depth=5, anomalies=anomalies)
    if shuffle:  # the job must not depend on storage order at all
        random.Random(seed).shuffle(spans)
    ids: dict = {}
    cols = to_columns(spans, ids)
    names = {v: k for k, v in ids.items()}
    S = max(len(ids), 1)
    r = oracle.aggregate(cols, S, threads=3)
    ref = aggregate_job(spans, strict=False)
    assert r.stats["ambiguous"] == 0
    assert r.stats["no_service"] == ref.no_service
    got = {(names[p], names[c]): m for (p, c), m in r.moments().items()}
    want = ref.exact()
    assert set(got) == set(want)
    for k in want:
        assert got[k] == want[k], k  # exact power sums -> identical rounding
        # and within the north-star tolerance of the reference's Algebird fold
        assert moments_close(algebird_fold(float(d) for d in ref.durations[k]), got[k]), k


def test_c_oracle_thread_count_invariant():
    from zipkin_amd import tracegen_host

    cols = tracegen_host(seed=5, num_traces=3000, max_depth=6, num_services=20)
    a = oracle.aggregate(cols, 20, threads=1)
    b = oracle.aggregate(cols, 20, threads=7)
    assert np.array_equal(a.cells, b.cells) and a.stats == b.stats


def test_c_oracle_record_order_invariant():
    from zipkin_amd import tracegen_host

    cols = tracegen_host(seed=6, num_traces=2000, max_depth=6, num_services=30)
    perm = np.random.default_rng(0).permutation(len(cols))
    a = oracle.aggregate(cols, 30)
    b = oracle.aggregate(cols.take(perm), 30)
    assert np.array_equal(a.cells, b.cells) and a.stats == b.stats


def test_moments_exact_vs_fold_on_tracegen_links():
    from zipkin_amd import tracegen_host

    cols = tracegen_host(seed=7, num_traces=500, max_depth=5, num_services=8)
    r = oracle.aggregate(cols, 8)
    for key, m in r.moments().items():
        assert m.m0 >= 1 and m.m2 >= 0 and m.m4 >= 0
