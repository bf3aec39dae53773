"""Rich-span workload for parity tests: TraceGen-shaped traces with real annotations
(TraceGen.scala:50-143), plus optional injected anomalies the reference's semantics must survive.
Test infrastructure only."""
from __future__ import annotations

import random
from typing import List, Optional

from oracle.spans import Annotation, BinaryAnnotation, Endpoint, Span

SERVICE_WORDS = (
    "vitae ipsum felis lorem magna dolor porta donec augue tortor auctor mattis ligula mollis aenean "
    "montes semper magnis rutrum turpis sociis lectus mauris congue libero rhoncus dapibus natoque "
    "gravida viverra egestas lacinia feugiat pulvinar accumsan sagittis ultrices praesent vehicula "
    "nascetur pharetra maecenas consequat ultricies ridiculus malesuada curabitur convallis facilisis "
    "hendrerit penatibus imperdiet tincidunt parturient adipiscing consectetur pellentesque"
).split()


def gen_traces(
    seed: int,
    traces: int,
    max_depth: int = 5,
    services: Optional[List[str]] = None,
    anomalies: float = 0.0,
) -> List[Span]:
    rnd = random.Random(seed)
    svcs = services or SERVICE_WORDS
    out: List[Span] = []

    def ep(name):
        return Endpoint(rnd.getrandbits(32), rnd.randrange(1000, 9000), name)

    def pick(upstream):
        for _ in range(len(svcs) + 1):
            s = rnd.choice(svcs)
            if s not in upstream:
                return s
        return rnd.choice(svcs)

    for _ in range(traces):
        tid = rnd.getrandbits(64) - 2**63
        spans: List[Span] = []
        upstream = []

        def do_rpc(t, depth, name, e, sid, pid):
            cur = t + 1000
            annos = [Annotation(cur, "sr", e)]
            bins = tuple(BinaryAnnotation(rnd.choice(svcs), b"v", "String", e) for _ in range(rnd.randint(1, 3)))
            cur += rnd.randrange(10) * 1000
            for _ in range(rnd.randint(2, 6)):
                annos.append(Annotation(cur, rnd.choice(svcs), e))
                cur += rnd.randrange(5) * 1000
            if depth > 0:
                times = []
                for _ in range(rnd.randint(2, depth + 1)):
                    child_svc = pick(upstream)
                    upstream.append(child_svc)
                    ce = ep(child_svc)
                    csid = rnd.getrandbits(64) - 2**63
                    delay = rnd.randrange(10) if rnd.randrange(10) > 6 else 0
                    cs = Annotation(cur + delay, "cs", ce)
                    ret = do_rpc(cur, rnd.randrange(depth), "rpc", ce, csid, sid) + 1000
                    spans.append(Span(tid, "rpc", csid, sid, (cs, Annotation(ret, "cr", ce)), ()))
                    upstream.pop()
                    times.append(ret)
                cur = max(times)
            annos.append(Annotation(cur, "ss", e))
            spans.append(Span(tid, name, sid, pid, tuple(annos), bins))
            return cur

        root_svc = pick(upstream)
        upstream.append(root_svc)
        do_rpc(1_400_000_000_000_000 + rnd.randrange(10**9), rnd.randrange(max_depth), "root", ep(root_svc),
               rnd.getrandbits(64) - 2**63, None)
        upstream.pop()
        if anomalies and rnd.random() < anomalies:
            spans = _inject(rnd, spans)
        out.extend(spans)
    return out


def _inject(rnd: random.Random, spans: List[Span]) -> List[Span]:
    kind = rnd.randrange(6)
    i = rnd.randrange(len(spans))
    s = spans[i]
    if kind == 0:  # duplicate a stored fragment -> doubled core annotations -> invalid span
        spans.append(s)
    elif kind == 1:  # lose a span -> its children miss their parent
        spans.pop(i)
    elif kind == 2:  # a span without any core-annotation host (no service) and no core annotations
        spans[i] = Span(s.trace_id, s.name, s.id, s.parent_id,
                        tuple(Annotation(a.timestamp, a.value, None) for a in s.annotations), s.binary_annotations)
    elif kind == 3:  # custom annotation far outside the core ones stretches the duration
        spans[i] = Span(s.trace_id, s.name, s.id, s.parent_id,
                        s.annotations + (Annotation(s.annotations[-1].timestamp + 77_777, "late", None),),
                        s.binary_annotations)
    elif kind == 4:  # self-parented span (every fragment of it, so the fragments still agree)
        spans = [Span(x.trace_id, x.name, x.id, x.id, x.annotations, x.binary_annotations) if x.id == s.id else x
                 for x in spans]
    else:  # shuffle the fragment order inside the trace (storage order is not guaranteed)
        rnd.shuffle(spans)
    return spans
