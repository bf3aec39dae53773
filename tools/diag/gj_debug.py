"""Diagnostic: one shuffled TraceGen batch through the group join of the loaded library vs P3 + K1
(zk_config.trace_pass = 1), printing the counters that differ and the m0 difference."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from zipkin_amd import DepsContext, tracegen_host  # noqa: E402


def run(cols, S, trace_pass=False):
    with DepsContext(S, trace_pass=trace_pass) as ctx:
        ctx.accumulate(cols, verify=False)
        return ctx.finalize(), ctx.stats()


traces = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000
S = 57
cols = tracegen_host(51, traces, max_depth=6, num_services=S)
sh = cols.take(np.random.default_rng(51).permutation(len(cols)))
got, sg = run(sh, S)
ref, sr = run(sh, S, trace_pass=True)
print("records", len(cols), "m0 sum", int(got.m0.sum()), int(ref.m0.sum()), "cells differing", int((got.m0 != ref.m0).sum()))
print({k: (sg[k], sr[k]) for k in sg if sg[k] != sr[k]})
