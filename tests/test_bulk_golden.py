"""Bulk job goldens: TraceGen-shaped batches of 1e3 / 1e4 / 1e5 traces with fixed
seeds, pinned in tests/golden/bulk_job.json (tools/make_golden.py --only bulk_job.json).

The CPU test pins the oracle (record / link / stat totals, SHA-256 of the exact per-cell power sums
and of the exactly rounded dense m0..m4); the GPU test pins the device's finalize output to the
same digest, bit for bit. Parity of the job arithmetic with the reference itself stays "unpinned"
(no reference output exists): these fixtures hold results across rounds."""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np
import pytest

from zipkin_amd import tracegen_host

ROOT = Path(__file__).resolve().parent.parent
GOLD = json.loads((ROOT / "tests" / "golden" / "bulk_job.json").read_text())["cases"]
sys.path.insert(0, str(ROOT / "tools"))


def _cols(case):
    return tracegen_host(seed=case["seed"], num_traces=case["traces"], max_depth=case["max_depth"],
                         num_services=case["services"])


@pytest.mark.parametrize("name", sorted(GOLD))
def test_oracle_bulk_golden(name):
    from make_golden import bulk_digests

    case = GOLD[name]
    got = bulk_digests(_cols(case), case["services"])
    for k in ("records", "links", "joined", "stats", "power_sums_sha256", "dense_moments_sha256"):
        assert got[k] == case[k], k


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GOLD))
def test_device_bulk_golden(name):
    from zipkin_amd import DepsContext

    case = GOLD[name]
    cols = _cols(case)
    with DepsContext(case["services"], device=0) as ctx:
        ctx.accumulate(cols)
        t = ctx.finalize()
        st = ctx.stats()
    dense = b"".join([np.ascontiguousarray(t.m0, dtype=np.uint64).tobytes()] +
                     [np.ascontiguousarray(m, dtype=np.float64).tobytes() for m in (t.m1, t.m2, t.m3, t.m4)])
    assert hashlib.sha256(dense).hexdigest() == case["dense_moments_sha256"]
    assert int(t.present.sum()) == case["links"]
    for k, v in case["stats"].items():
        assert st[k] == v, k
