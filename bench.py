#!/usr/bin/env python3
"""Headline benchmark: spans/sec into DependencyLinks (+ % of HBM roofline), BASELINE.json.

One step = one pass of the zipkin-aggregate dependency path over one batch already resident in
HBM: reset the exact accumulator, accumulate the batch (K1 span_join + spill), [N>1: RCCL SUM
all-reduce of the accumulator across traceId-hash shards], finalize into device-resident
(parent, child) -> Moments arrays (K5), including the status check the reference's fail-fast
semantics need.

Workloads (synthetic, zipkin-tracegen shape: maxDepth 6, ~24 records / ~12 logical spans per trace,
500 services, generated on device):
  C2 (default at N = 1, BASELINE.json configs[1]): 1e8 span records on one GPU.
  C3 (default at N > 1, configs[2]): ONE global set of 1e9 span records whose traceIds do not depend
     on N, sharded by mix64(traceId) % N -- rank r generates exactly the set's traces of its shard --
     with one RCCL SUM all-reduce of the exact table per step (strong scaling: the same 1e9 records
     at every N). Every rank hashes the finalized table (SHA-256 of m0..m4 + present); the digests
     must agree across ranks and with the G = 1 digest in tests/golden/c3_digest.json.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.3 TB/s is the measured copy rate
BYTES_PER_RECORD = 48


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--records", type=int, default=None,
                    help="c2: span records per GPU (default 1e8); c3: records of the whole global set (default 1e9)")
    ap.add_argument("--services", type=int, default=500)
    ap.add_argument("--max-depth", type=int, default=6)
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--cpu-sample", type=int, default=100_000_000,
                    help="records for the CPU baseline and oracle parity leg (0: skip; default: the whole C2 batch)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: every CPU this process may use, see usable_cpus)")
    ap.add_argument("--verify", type=int, default=0,
                    help="1: ZK_BATCH_VERIFY_TRACES on every step (exact device check of the clustering promise)")
    ap.add_argument("--pipeline", type=int, default=None,
                    help="batches in flight behind the one being joined: 1 = two table/stream "
                         "sets (batch k's join overlaps batch k-1's tail), 2 = three, 0 = one set, serial steps "
                         "(c2/c3 take any depth, c4/c5 use two sets when > 0). Default: 3 for c2/c3 (four sets: "
                         "1.447-1.448 ms per C2 step against 1.500-1.518 with two, same box, "
                         "profiles/r04/ab_pipeline_depth.txt), 1 for c5, 0 for c4, whose partition scatter and "
                         "candidate pass each fill the LDS of a CU, so two overlapped sets only contend "
                         "(12.06 ms serial vs 14.13 ms pipelined, profiles/r02/ab_c4_pipeline.txt)")
    ap.add_argument("--overlap", default="full", choices=("tail", "full"),
                    help="c2 pipelined steps: full (default) = no ordering between the table sets: batch k's "
                         "join shares the GPU with batch k-1's K2/K3 (faster steps; K1's launch events then also "
                         "cover the K2/K3 work it shares the chip with, see roofline.isolated_*); tail = batch k's "
                         "join starts once batch k-1's reduce is done, so only spill, [all-reduce,] finalize, "
                         "status check and reset overlap the next join and every K1 launch runs alone")
    ap.add_argument("--order", default="clustered", choices=("clustered", "shuffled"),
                    help="c2: clustered (default) = the batch as TraceGen emits it, trace-clustered like "
                         "Cassandra row-per-trace reads, accumulated with ZK_BATCH_TRACE_CLUSTERED; shuffled = "
                         "the same records in a random permutation (the reference's shuffles accept any order, "
                         "ZipkinAggregateJob.scala:21-22,28-33): every step runs the device clustering pass first")
    ap.add_argument("--workload", default=None, choices=("c1", "c2", "c3", "c4", "c5", "ingest"),
                    help="default: c2 at N = 1, c3 at N > 1. c2 (the N = 1 headline): dependency path on 1e8 "
                         "records; c3: the same path on one global 1e9-record set sharded across the N ranks "
                         "(configs[2]); c1: the reference's CPU config "
                         "(10k tracegen traces, 20 services) on the GPU and the CPU baseline; "
                         "c4: key-value top-K sketch over "
                         "binary annotations; c5: per-service HLL + duration histogram from span fragments; "
                         "ingest: device decode of stored Snappy+thrift fragments into columns")
    ap.add_argument("--fragments", type=int, default=20_000_000, help="ingest: stored fragments per step")
    ap.add_argument("--ingest-items", type=int, default=0,
                    help="ingest: 1 = decode with the span indexer's items (zk_ingest_dev_spans_items), checked "
                         "against the host decoder's items as a multiset per replica")
    ap.add_argument("--ingest-batches", type=int, default=1,
                    help="ingest: the step's fragments as this many separate stored batches (separate tensors), "
                         "decoded by ONE zk_ingest_dev_spans_multi call per step; the line's detail also times "
                         "one decode call per batch")
    ap.add_argument("--comm", default=None, choices=("zk", "torch"),
                    help="N > 1: the exchange's collective. zk (default with RCCL) = the library's own "
                         "communicator, zk_deps_allreduce / zk_rt_allreduce (include/zkcomm.h), the call the "
                         "JVM drop-in makes (GpuDependenciesJob.scala); torch = torch.distributed all_reduce "
                         "of the same exchange buffer (default for the gloo rehearsal, where RCCL cannot run "
                         "two ranks on one GPU)")
    ap.add_argument("--layout", default="separate", choices=("separate", "packed"),
                    help="c2/c3: the device columns as seven allocations (separate) or back to back in one "
                         "(packed, DeviceColumns(packed=True))")
    ap.add_argument("--items", type=int, default=1_000_000_000,
                    help="c4: binary annotations per step (BASELINE configs[3]: 1e9, 12 GB in HBM)")
    a = ap.parse_args()
    if a.workload is None:
        a.workload = "c3" if int(os.environ.get("WORLD_SIZE", "1")) > 1 else "c2"
    if a.records is None:  # c3 and c5 run configs[2] / configs[4] at their stated 1e9 spans
        a.records = 1_000_000_000 if a.workload in ("c3", "c5") else 100_000_000
    if a.pipeline is None:
        a.pipeline = 3 if a.workload in ("c2", "c3") else 0 if a.workload == "c4" else 1
    if a.comm is None:
        a.comm = "zk" if os.environ.get("ZK_BENCH_BACKEND", "nccl") == "nccl" else "torch"
    return a


def init_dist():
    """(world, rank, local, dist or None): one process per GPU, RANK/LOCAL_RANK/WORLD_SIZE from the
    launcher; ZK_BENCH_BACKEND=gloo is the correctness rehearsal with several ranks on one GPU."""
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1:
        torch.cuda.set_device(0)
        return 1, 0, 0, None
    import torch.distributed as dist

    backend = os.environ.get("ZK_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return world, rank, local, dist


def zk_comms(dist, rank, world, local, count):
    """`count` communicators of the library (include/zkcomm.h), one per table/stream set: rank 0 makes
    the RCCL unique ids, torch.distributed's bootstrap hands them to the other ranks (the JVM host does
    the same over its own channel), every rank opens them in the same order."""
    from zipkin_amd.comm import Comm, unique_id

    ids = [[unique_id() for _ in range(count)] if rank == 0 else None]
    dist.broadcast_object_list(ids, src=0)
    return [Comm(u, rank, world, device=local) for u in ids[0]]


def main():
    a = parse()
    import torch

    if a.workload == "c1":
        return bench_c1(a)
    if a.workload == "c4":
        return bench_c4(a)
    if a.workload == "c5":
        return bench_c5(a)
    if a.workload == "ingest":
        return bench_ingest(a)

    # ZK_BENCH_BACKEND=gloo: a correctness rehearsal of the N>1 path with several ranks on one GPU
    # (not a measurement); the driver's runs use RCCL, one rank per GPU
    world, rank, local, dist = init_dist()
    dev = torch.device("cuda", local)

    from zipkin_amd import DepsContext, DeviceColumns, tracegen_params
    from zipkin_amd.shards import allreduce_table, device_view

    c3 = a.workload == "c3"
    S = a.services
    cells = S * S
    # one dedicated stream orders the library's kernels, torch's allocations and RCCL (a handle of
    # 0 -- torch's legacy default stream -- would make the library create an unordered private one)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    ctx = DepsContext(S, device=local, stream=stream.cuda_stream, timing=True)
    traces_cap = int(a.records / 15) + 1000
    if c3:
        # one global set of a.records records: this rank generates the set's traces of its shard
        p = tracegen_params(a.seed, traces_cap, target_records=a.records, max_depth=a.max_depth, num_services=S,
                            rank=rank, world=world, global_ids=True)
        cap = int(a.records / world * 1.02) + 1_000_000  # shards are hash-balanced (+-0.1 % at 4e7 traces)
    else:
        p = tracegen_params(a.seed, traces_cap, target_records=a.records, max_depth=a.max_depth, num_services=S,
                            rank=rank, world=world)
        cap = a.records
    cols = DeviceColumns(cap, device=f"cuda:{local}", packed=a.layout == "packed")
    n, ntr = ctx.tracegen_device(p, cols)
    total_hint = n * world  # records of the whole job per step (exact below, before the timed steps)
    if dist is not None:
        tt = torch.tensor([n], dtype=torch.int64, device=dev)
        dist.all_reduce(tt)
        total_hint = int(tt.item())
    shuffled = a.order == "shuffled"
    clustered_cols = cols
    if shuffled:
        # the same records in a random order, permuted once before the timed region
        g = torch.Generator(device=dev)
        g.manual_seed(a.seed + 1000 * rank)
        perm = torch.randperm(n, device=dev, generator=g)
        sc = DeviceColumns(n, device=f"cuda:{local}", packed=a.layout == "packed")
        for k in ("trace_id", "span_id", "parent_id", "first_ts", "last_ts", "service_id", "flags"):
            torch.index_select(getattr(cols, k)[:n], 0, perm, out=getattr(sc, k))
        # the gathers run on `stream`; the second table set's context later writes memory torch may
        # recycle from `perm` on ANOTHER stream, so the gathers must be done before perm is released
        torch.cuda.synchronize()
        del perm
        cols = sc
    out = {
        "m0": torch.empty(cells, dtype=torch.int64, device=dev),
        "m1": torch.empty(cells, dtype=torch.float64, device=dev),
        "m2": torch.empty(cells, dtype=torch.float64, device=dev),
        "m3": torch.empty(cells, dtype=torch.float64, device=dev),
        "m4": torch.empty(cells, dtype=torch.float64, device=dev),
        "present": torch.empty(cells, dtype=torch.uint8, device=dev),
    }

    nsets = (a.pipeline + 1) if a.pipeline != 0 else 1
    comms, comm_note = None, None
    if dist is not None and a.comm == "zk":
        try:
            comms = zk_comms(dist, rank, world, local, nsets)
        except Exception as e:  # reported in the line; the same exchange then goes through torch
            comm_note = f"zk_comm_create failed ({e}); torch.distributed all_reduce used instead"
            print(f"[bench] {comm_note}", file=sys.stderr, flush=True)
            comms = None
        ok = torch.tensor([1 if comms is not None else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)  # every rank takes the same path
        if int(ok.item()) == 0 and comms is not None:
            for cm in comms:
                cm.close()
            comms = None
            comm_note = comm_note or "zk_comm_create failed on another rank; torch.distributed all_reduce used instead"
    ar_events = []  # (start, end) HIP events around the all-reduce of the serial warmup steps

    def exchange(c, s, i, timed=False):
        """N > 1: the merge of the ranks' tables (ZipkinAggregateJob.scala:39-43 .group.sum / .sum), on
        the set's stream s, after its accumulate and before its finalize."""
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
        if comms is not None:
            # zk_deps_allreduce: partial (counters folded, 56-bit limbs) -> RCCL int64 SUM -> note_merged
            comms[i].allreduce_deps(c, total_hint)
        else:
            xp, xb = c.partial()
            # the same exact limb + counter SUM through torch.distributed
            allreduce_table(device_view(xp, xb, torch.int64, local))
            c.note_merged(total_hint)
        if timed:
            e1.record(s)
            ar_events.append((e0, e1))

    def step_serial():
        ctx.reset()
        # device-generated batches are trace-clustered by construction (zk_tracegen_device)
        ctx.accumulate(cols, clustered=not shuffled, verify=a.verify)
        if dist is not None:
            exchange(ctx, stream, 0, timed=True)
        ctx.finalize(out_device=out)

    step = step_serial

    def drain():
        pass

    pipeline = a.pipeline != 0
    if pipeline:
        # a.pipeline + 1 table/stream sets, software-pipelined: batch k's join runs on its stream while
        # earlier batches' tails (K2/K3, at N > 1 the all-reduce over RCCL, finalize and status check)
        # complete on the others; every batch is still joined, reduced and finalized inside the timed
        # region (drain() finalizes the last ones).
        sets = [(ctx, None, stream, out)]
        for _ in range(a.pipeline):  # a.pipeline batches in flight behind the one being joined
            s2 = torch.cuda.Stream(device=dev)
            c2 = DepsContext(S, device=local, stream=s2.cuda_stream, timing=False)
            sets.append((c2, None, s2, {k: torch.empty_like(v) for k, v in out.items()}))
        state = {"k": 0, "pending": []}

        def finalize_oldest():
            pc, _, ps, po = state["pending"].pop(0)
            torch.cuda.set_stream(ps)
            pc.finalize(out_device=po)

        def step():  # noqa: F811
            i = state["k"] % len(sets)
            c, t, s, o = sets[i]
            state["k"] += 1
            torch.cuda.set_stream(s)
            c.reset()
            if a.overlap == "tail" and state.get("reduced") is not None:
                s.wait_event(state["reduced"])  # K1 after the previous batch's K2/K3
            c.accumulate(cols, clustered=not shuffled, verify=a.verify)
            if a.overlap == "tail":
                ev = torch.cuda.Event()
                ev.record(s)
                state["reduced"] = ev
            if dist is not None:
                exchange(c, s, i)  # ordered on s; the host does not wait
            state["pending"].append((c, t, s, o))
            if len(state["pending"]) > a.pipeline:
                finalize_oldest()

        def drain():  # noqa: F811
            while state["pending"]:
                finalize_oldest()
            torch.cuda.set_stream(stream)

    debug = os.environ.get("ZK_BENCH_DEBUG") == "1"

    def csum(c):
        return [int(getattr(c, k)[:n].to(torch.int64).sum().item()) for k in
                ("trace_id", "span_id", "parent_id", "first_ts", "last_ts", "service_id", "flags")]

    if debug:
        sums0 = (csum(cols), csum(clustered_cols))
    # warmup: serial steps first (their K1 launches give the isolated K1 duration), then two
    # pipelined steps so that the second set's buffers exist before the timed region
    # (at least ISOLATED + 1 serial steps: untimed, outside the timed region, so that the isolated K1
    # figure averages several warm launches whatever --warmup is)
    ISOLATED = 8
    tmf = None
    for i in range(max(a.warmup, ISOLATED + 1)):
        step_serial()
        if i == 0:  # the first launch is cold: the isolated figure averages the later ones
            tmf = dict(ctx.timing())
    torch.cuda.synchronize()
    tmw = ctx.timing()
    k1_isolated_ms = (tmw["join_ms_total"] - tmf["join_ms_total"]) / (tmw["join_calls"] - tmf["join_calls"])
    isolated_launches = tmw["join_calls"] - tmf["join_calls"]
    if pipeline:
        for _ in range(len(sets)):
            step()
        drain()
    torch.cuda.synchronize()
    tm0 = ctx.timing()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(a.steps):
        step()
    drain()
    if pipeline:
        for st2 in sets[1:]:
            stream.wait_stream(st2[2])
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    tm1 = ctx.timing()
    ev_ms = ev0.elapsed_time(ev1)
    elapsed = wall
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total_records = total_hint  # the records every rank actually aggregated (shards differ in size)
    allreduce_ms = None
    if ar_events:
        ms = [e0.elapsed_time(e1) for e0, e1 in ar_events[1:]] or [ar_events[0][0].elapsed_time(ar_events[0][1])]
        allreduce_ms = sorted(ms)[len(ms) // 2]
    value = total_records * a.steps / elapsed
    join_calls = tm1["join_calls"] - tm0["join_calls"]
    join_avg_ms = (tm1["join_ms_total"] - tm0["join_ms_total"]) / max(1, join_calls)
    st = ctx.stats()
    if pipeline:
        # both pipeline sets finalized the same batch: their outputs must agree bit for bit
        for c2, _, _, o2 in sets[1:]:
            for k in out:
                if not torch.equal(out[k], o2[k]):
                    raise RuntimeError(f"pipelined step: output '{k}' differs between the table sets")
            c2.close()

    # the finalized table's digest on every rank (all ranks hold the merged job): C3 checks it
    # against the other ranks and against the G = 1 digest of the same global set
    digest = table_digest(out)
    digest_check = None
    if c3:
        digests = [digest]
        if dist is not None:
            digests = [None] * world
            dist.all_gather_object(digests, digest)
        if len(set(digests)) != 1:
            raise RuntimeError(f"C3: the ranks' finalized tables differ: {digests}")
        key = f"seed{a.seed}_records{a.records}_S{S}_depth{a.max_depth}"
        golden = ROOT / "tests" / "golden" / "c3_digest.json"
        gd = json.loads(golden.read_text()) if golden.exists() else {}
        want = gd.get(key, {}).get("sha256")
        if want is not None and want != digest:
            raise RuntimeError(f"C3 at N = {world}: table digest {digest} != the G = 1 digest {want} ({golden})")
        digest_check = {"sha256": digest, "ranks_agree": True,
                        "vs_g1": ("exact" if want == digest else "no G = 1 digest recorded for this set"),
                        "golden": f"tests/golden/c3_digest.json[{key}]"}
    if debug:
        sums1 = (csum(cols), csum(clustered_cols))
        print(f"[debug] column sums before/after: {sums0 == sums1} {sums0} {sums1}", file=sys.stderr, flush=True)
    cpu = parity = None
    shuffled_parity = None
    if shuffled:
        # the whole shuffled batch must give the clustered batch's result bit for bit (every cell's
        # m0..m4 and every counter): permutation invariance at full size
        ref_out = {k: torch.empty_like(v) for k, v in out.items()}
        with DepsContext(S, device=local, stream=stream.cuda_stream) as cref:
            cref.accumulate(clustered_cols, clustered=True, verify=False, n=n)
            cref.finalize(out_device=ref_out)
            stc = cref.stats()
        bad = [k for k in out if not torch.equal(out[k], ref_out[k])]
        bad += [k for k, v in stc.items() if k != "spilled_traces" and st[k] != v]
        if bad:
            ncell = int((out["m0"] != ref_out["m0"]).sum())
            raise RuntimeError(f"shuffled batch differs from the clustered batch: {bad}; {ncell} cells differ in m0; "
                               f"shuffled stats {st}, clustered stats {stc}")
        shuffled_parity = {"result": "exact", "records": n,
                           "checked": "m0..m4, present and all counters of the shuffled full batch == the clustered batch"}
    full = None
    if rank == 0 and world == 1 and c3 and a.cpu_sample > 0:
        # configs[2] pinned at full size: the CPU port over the WHOLE global set, bit for bit
        cpu, full = c3_full_oracle(clustered_cols, n, S, a.cpu_threads or usable_cpus(), out, st, digest)
    elif rank == 0 and world == 1 and a.cpu_sample > 0 and shuffled:
        # the shuffled batch as it is (any order: no prefix of it is trace-complete) through the port's
        # hash-partitioned mode, against the GPU's table of the same batch
        cpu, parity = shuffled_oracle(cols, n, S, a.cpu_threads or usable_cpus(), out, st)
    elif rank == 0 and world == 1 and a.cpu_sample > 0:
        cpu, parity = cpu_baseline(clustered_cols, min(a.cpu_sample, n), S, a.cpu_threads or usable_cpus(), dev)
    if c3:
        parity = {"digest": digest_check, "full_vs_oracle": full, "prefix_vs_oracle": parity}

    # PMC counters need their own rocprofv3 --pmc run (tools/pmc.sh), so the traffic figure is the
    # builder's measurement of the same kernel on the same workload, labelled with its source
    traffic = traffic_src = None
    pmc = ROOT / "profiles" / "pmc_latest.json"
    if pmc.exists():
        try:
            j = json.loads(pmc.read_text())
            if j.get("records") == n:
                traffic = j.get("hbm_bytes_per_launch")
                traffic_src = f"profiles/pmc_latest.json ({j.get('run', 'builder run')}, rocprofv3 --pmc, not this run)"
        except Exception:
            traffic = None

    if rank == 0:
        line = {
            "metric": "spans/sec into DependencyLinks (1/2/4/8 GPU) + % of HBM roofline",
            "value": value,
            "unit": "spans/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": "strong" if c3 else "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (zipkin-tracegen-shaped, generated on device)",
            "config": {
                "workload": (f"C3: one global set of {a.records:.3g} span records (BASELINE configs[2]) sharded by "
                             f"mix64(traceId) % {world} across {world} GPU(s), {S} services, dependency link table + "
                             "Moments, RCCL SUM all-reduce of the exact table" if c3 else
                             "C2: 1e8 span records/GPU, 500 services, dependency link table + Moments")
                            + (" (records in random order: device clustering pass in every step)" if shuffled else ""),
                "total_records": total_records,
                "records_per_gpu": n,
                "traces_per_gpu": ntr,
                "records_per_trace": round(n / max(1, ntr), 2),
                "vs_configs_1": "BASELINE configs[1] names 100M spans / 5M traces (20 records per trace); TraceGen "
                                "with integer maxDepth gives 15.2 (depth 5) or 24.1 (depth 6) records per trace, so "
                                f"the batch holds {n:.3g} records in {ntr:.3g} whole traces (maxDepth {a.max_depth})",
                "services": S,
                "max_depth": a.max_depth,
                "parallelism": f"traceId-hash shards x{world}" + (", RCCL all-reduce of the link table" if world > 1 else ""),
                "collective": (None if world == 1 else
                               "zk_deps_allreduce: libzkagg's own RCCL communicator (include/zkcomm.h), the JVM "
                               "drop-in's call" if comms is not None else
                               f"torch.distributed all_reduce ({os.environ.get('ZK_BENCH_BACKEND', 'nccl')}) of "
                               "zk_deps_partial's exchange buffer" + (f" -- {comm_note}" if comm_note else "")),
                "step": "reset + span_join + spill + [all-reduce] + finalize(m0..m4) + status check"
                        + ((f" ({a.pipeline + 1} table sets: batch k's join follows batch k-1's reduce and overlaps "
                            "its [all-reduce,] finalize, status check and reset)") if pipeline and a.overlap == "tail" else
                           (f" ({a.pipeline + 1} table sets: batch k's join overlaps earlier batches' reduce, [all-reduce,] "
                            "finalize)") if pipeline else ""),
            },
            # K1 (the dominant kernel) timed ALONE: HIP events on the ctx stream around each K1 launch
            # of the serial steps (nothing else on the chip: no overlap with the other table set's
            # K2/K3), averaged over `launches` warm launches -- the figure rocprofv3's serial kernel
            # stats reproduce. The pipelined launches of the timed steps share the chip with the other
            # set's reduce, so their event spans are not a kernel duration: detail.pipelined_k1_*.
            "roofline": {
                "bound": "hbm",
                "kernel": ("k_group_join (+ the fallback's P3 list pass and K1 append, normally empty)"
                           if shuffled and not a.verify else "k_span_join_stream"),
                "achieved": n * BYTES_PER_RECORD / (k1_isolated_ms * 1e-3) / 1e9,
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": n * BYTES_PER_RECORD / (k1_isolated_ms * 1e-3) / 1e9 / PEAK_HBM_GBS,
                "traffic": traffic if not shuffled else None,
                "traffic_source": traffic_src if not shuffled else None,
                "algorithmic_bytes_per_launch": n * BYTES_PER_RECORD,
                "bytes_per_record": BYTES_PER_RECORD,
                "avg_launch_ms": k1_isolated_ms,
                "launches": isolated_launches,
                "timing": "HIP events on the ctx stream around each join launch of serial (non-overlapped) steps",
                # the whole step's algorithmic bytes (K1's input) over the step time
                "step_frac": n * BYTES_PER_RECORD / (elapsed / a.steps) / 1e9 / PEAK_HBM_GBS,
            },
            "cpu_baseline": cpu,
            "parity": parity if not shuffled else {"full_vs_oracle": parity, "shuffled_vs_clustered": shuffled_parity},
            "detail": {
                "event_ms_per_step": ev_ms / a.steps,
                # N > 1: the exchange alone (partial + collective + note_merged), HIP events on the ctx
                # stream around it in the serial warmup steps, median (24 MB int64 SUM at S = 500)
                "allreduce_ms": allreduce_ms,
                # K1 event spans inside the timed (pipelined) steps: they also cover the other table
                # set's K2/K3 that share the chip with K1, so they are longer than the kernel
                "pipelined_k1_event_ms": join_avg_ms,
                "pipelined_k1_launches": join_calls,
                "order": a.order,
                "cluster_ms_avg": ((tm1["cluster_ms_total"] - tm0["cluster_ms_total"]) / max(1, join_calls)
                                   if shuffled else 0.0),
                "finalize_ms_last": tm1["finalize_ms"],
                "reduce_avg_ms": (tm1["reduce_ms_total"] - tm0["reduce_ms_total"]) / max(1, join_calls),
                "spill_ms_last": tm1["spill_ms"],
                "joined_links_per_step": int(st["joined_links"]),  # stats cover the last step (reset per step)
                "merged_spans_per_step": int(st["merged_spans"]),
                "merged_spans_per_s": int(st["merged_spans"]) * world * a.steps / elapsed,
            },
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    for cm in comms or ():
        cm.close()
    if dist is not None:
        dist.destroy_process_group()


def table_digest(out) -> str:
    """SHA-256 of a finalized table (m0 u64, m1..m4 f64, present u8, in that order, cell-major)."""
    import hashlib

    h = hashlib.sha256()
    for k in ("m0", "m1", "m2", "m3", "m4", "present"):
        h.update(out[k].cpu().numpy().tobytes())
    return h.hexdigest()


def usable_cpus() -> int:
    """CPUs this process may run on: its affinity mask, capped by a cgroup CPU quota and by the
    thread budget the box exports (OMP_NUM_THREADS), whichever is smallest."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()
        if q != "max":
            n = min(n, max(1, int(q) // int(per)))
    except Exception:
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        n = min(n, int(omp))
    return max(1, n)


def cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def c3_full_oracle(cols, n, S, threads, out, st, digest):
    """configs[2] at G = 1 against the oracle at full size: the whole global set (1e9 records) copied
    to the host and aggregated by oracle/zk_cpu_port.c (trace-clustered pass, bit-identical to the
    literal oracle/zk_oracle.c by tests/test_cpu_port.py) on every usable core; its m0..m4, present
    and counters must equal the GPU's finalized table and stats bit for bit, else the bench fails.
    The oracle's table digest is what tests/golden/c3_digest.json records. The port's time over the
    whole set is the C3 line's CPU baseline (kind "port")."""
    import numpy as np

    from oracle import oracle

    t0 = time.perf_counter()
    host = cols.to_host(n)
    copy_s = time.perf_counter() - t0
    rp = oracle.aggregate_port(host, S, threads=threads, clustered=True)
    m0, ms = rp.dense()
    ref = {"m0": m0.view(np.int64), "m1": ms[0], "m2": ms[1], "m3": ms[2], "m4": ms[3],
           "present": (m0 > 0).astype(np.uint8)}
    bad = [k for k in ref if not np.array_equal(out[k].cpu().numpy(), ref[k])]
    bad += [k for k, v in rp.stats.items() if k != "spilled_traces" and st[k] != v]
    if bad:
        raise RuntimeError(f"C3: the GPU table differs from oracle/zk_cpu_port.c over the whole set: {bad}")
    import hashlib

    h = hashlib.sha256()
    for k in ("m0", "m1", "m2", "m3", "m4", "present"):
        h.update(np.ascontiguousarray(ref[k]).tobytes())
    odig = h.hexdigest()
    if odig != digest:
        raise RuntimeError(f"C3: oracle digest {odig} != GPU digest {digest}")
    del host
    cpu = {"value": n / rp.seconds, "unit": "spans/s", "cores": threads, "kind": "port", "cpu": cpu_model(),
           "sample": f"the whole set ({n} records), oracle/zk_cpu_port.c (trace-clustered single pass), "
                     f"{threads} threads, one run: {rp.seconds:.2f} s (device-to-host copy {copy_s:.1f} s not counted)"}
    full = {"result": "exact", "records": n, "links": int((m0 > 0).sum()), "oracle_sha256": odig,
            "checked": "m0..m4, present and all counters of the GPU's finalized table == oracle/zk_cpu_port.c "
                       "over every record of the global set"}
    return cpu, full


def shuffled_oracle(cols, n, S, threads, out, st):
    """The shuffled line's parity leg and CPU baseline: the whole shuffled batch copied to the host and
    aggregated by oracle/zk_cpu_port.c in its hash-partitioned mode (any record order; bit-identical
    to oracle/zk_oracle.c by tests/test_cpu_port.py); its m0..m4, present and counters must equal the
    GPU's finalized table of the same batch, else the bench fails. The port's time is the baseline."""
    import numpy as np

    from oracle import oracle

    host = cols.to_host(n)
    rp = oracle.aggregate_port(host, S, threads=threads, clustered=False)
    m0, ms = rp.dense()
    ref = {"m0": m0.view(np.int64), "m1": ms[0], "m2": ms[1], "m3": ms[2], "m4": ms[3],
           "present": (m0 > 0).astype(np.uint8)}
    bad = [k for k in ref if not np.array_equal(out[k].cpu().numpy(), ref[k])]
    bad += [k for k, v in rp.stats.items() if k != "spilled_traces" and st[k] != v]
    if bad:
        raise RuntimeError(f"shuffled batch: the GPU table differs from oracle/zk_cpu_port.c: {bad}")
    cpu = {"value": n / rp.seconds, "unit": "spans/s", "cores": threads, "kind": "port", "cpu": cpu_model(),
           "sample": f"the whole shuffled batch ({n} records in random order), oracle/zk_cpu_port.c hash-partitioned "
                     f"mode, {threads} threads, one run: {rp.seconds:.2f} s"}
    parity = {"result": "exact", "records": n, "links": int((m0 > 0).sum()),
              "checked": "m0..m4, present and all counters of the shuffled batch's GPU table == oracle/zk_cpu_port.c "
                         "(hash-partitioned, any order) over the whole batch"}
    return cpu, parity


def cpu_baseline(cols, sample, S, threads, dev):
    """The CPU baseline (kind "port"): oracle/zk_cpu_port.c -- the same job as one multithreaded
    pass over trace-clustered input, the promise the GPU path runs under -- on the first `sample`
    records of the same batch, on this box's host cores. A reported baseline only.

    The literal oracle (oracle/zk_oracle.c) runs on the same prefix as the bench's parity check:
    the HIP path aggregates that prefix of the device batch, and m0..m4 and every counter must equal
    the oracle's bit for bit (and so must the port's), or the bench fails (the timed steps above
    process the full batch with the same kernels)."""
    import numpy as np

    from oracle import oracle
    from zipkin_amd import DepsContext

    host = cols.to_host(sample + 100_000)
    # cut at a trace boundary so the sample is trace-complete
    tid = host.trace_id
    cut = sample
    while cut < len(tid) and cut > 0 and tid[cut] == tid[cut - 1]:
        cut -= 1
    part = host.take(slice(0, cut))
    oracle.aggregate_port(part.take(slice(0, min(cut, 100_000))), S, threads=threads)  # warm the library
    times = []
    for _ in range(3):
        rp = oracle.aggregate_port(part, S, threads=threads, clustered=True)
        times.append(rp.seconds)
    port_s = sorted(times)[1]
    r = oracle.aggregate(part, S, threads=threads)
    if not (np.array_equal(rp.cells, r.cells) and rp.stats == r.stats):
        raise RuntimeError("the CPU port disagrees with the oracle")
    with DepsContext(S, device=dev.index or 0) as ctx:
        ctx.accumulate(cols, clustered=True, verify=True, n=cut)
        got = ctx.finalize()
        st = ctx.stats()
    m0, ms = r.dense()
    bad = [k for k, x, y in zip(("m0", "m1", "m2", "m3", "m4"), (got.m0, got.m1, got.m2, got.m3, got.m4), (m0, *ms))
           if not np.array_equal(x, y)]
    bad += [k for k, v in r.stats.items() if k != "spilled_traces" and st[k] != v]
    if bad:
        raise RuntimeError(f"parity failure on the {cut}-record prefix of the bench batch: {bad}")
    cpu = {
        "value": cut / port_s,
        "unit": "spans/s",
        "cores": threads,
        "kind": "port",
        "cpu": cpu_model(),
        "sample": f"first {cut} records (whole traces) of the benchmark batch; oracle/zk_cpu_port.c "
        f"(trace-clustered single pass), {threads} threads, median of 3: {port_s:.3f} s; the literal "
        f"oracle/zk_oracle.c took {r.seconds:.2f} s",
    }
    parity = {"result": "exact", "records": cut, "links": int(got.present.sum()),
              "checked": "m0..m4 bit-identical + all counters, HIP path vs oracle/zk_oracle.c, same prefix"}
    return cpu, parity


def _timed(step, steps, warmup, stream, others=()):
    import torch

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        step()
    for o in others:  # pipelined sets: the end event follows every stream's last step
        stream.wait_stream(o)
    ev1.record(stream)
    torch.cuda.synchronize()
    return time.perf_counter() - t0, ev0.elapsed_time(ev1)


def _thrift_fragments(cols, S):
    """Stored fragments for the ingest workload: one TBinaryProtocol Span per tracegen record
    (zipkinCore.thrift:50-58; core annotations with the record's service host, one custom
    annotation, one binary annotation), Snappy-compressed as CassieSpanStore stores them."""
    import struct

    import pyarrow as pa

    snappy = pa.Codec("snappy")

    def fh(t, i):
        return struct.pack(">bh", t, i)

    def st(b):
        return struct.pack(">i", len(b)) + b

    def ep(name, fid=3):  # Annotation.host is field 3, BinaryAnnotation.host field 4
        return fh(12, fid) + fh(8, 1) + struct.pack(">i", 0x7F000001) + fh(6, 2) + struct.pack(">h", 9410) + fh(11, 3) + st(name) + b"\0"

    def ann(ts, v, name):
        return fh(10, 1) + struct.pack(">q", ts) + fh(11, 2) + st(v) + (ep(name) if name else b"") + b"\0"

    out = []
    for i in range(len(cols)):
        f = int(cols.flags[i])
        name = b"service-%d" % int(cols.service_id[i])
        first, last = int(cols.first_ts[i]), int(cols.last_ts[i])
        core = (b"sr", b"ss") if f & 8 else (b"cs", b"cr")
        anns = [ann(first, core[0], name), ann((first + last) // 2, b"custom.event", name), ann(last, core[1], name)]
        body = fh(10, 1) + struct.pack(">Q", int(cols.trace_id[i])) + fh(11, 3) + st(b"rpc")
        body += fh(10, 4) + struct.pack(">Q", int(cols.span_id[i]))
        if f & 1:
            body += fh(10, 5) + struct.pack(">Q", int(cols.parent_id[i]))
        body += fh(15, 6) + struct.pack(">bi", 12, len(anns)) + b"".join(anns)
        body += fh(15, 8) + struct.pack(">bi", 12, 1) + fh(11, 1) + st(b"http.uri") + fh(11, 2) + st(b"/api/v1")
        body += fh(8, 3) + struct.pack(">i", 6) + ep(name, 4) + b"\0"
        body += fh(2, 9) + b"\0" + b"\0"
        out.append(snappy.compress(body, asbytes=True))
    return out


def bench_ingest(a):
    """The job's input decode on the device: stored Snappy(thrift Span)
    fragments already in HBM -> the 48-B columns (zk_ingest_dev). Fragments are synthesised on the
    host from tracegen records (a 200k-fragment set, replicated on the device to --fragments)."""
    import numpy as np
    import torch

    from zipkin_amd import tracegen_host
    from zipkin_amd.ingest import DeviceSpanDecoder, SpanDecoder

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    base = tracegen_host(a.seed, 9000, max_depth=a.max_depth, num_services=a.services)
    blobs = _thrift_fragments(base, a.services)
    m = len(blobs)
    reps = max(1, a.fragments // m)
    n = m * reps
    lens = np.array([len(b) for b in blobs], np.int64)
    one = torch.from_numpy(np.frombuffer(b"".join(blobs), np.uint8).copy()).to(dev)
    buf = one.repeat(reps)
    offs = np.zeros(n + 1, np.int64)
    offs[1:] = np.cumsum(np.tile(lens, reps))
    off = torch.from_numpy(offs).to(dev)
    in_bytes = int(offs[-1])
    dec = DeviceSpanDecoder(max(4096, a.services), stream=stream.cuda_stream)
    cols = None
    items = None
    # --ingest-batches K: the same fragments as K stored batches (views of the buffer, offsets rebased
    # per batch), as a job reading row batches holds them
    K = max(1, a.ingest_batches)
    cuts = [n * k // K for k in range(K + 1)]
    parts = [(buf[int(offs[lo]):int(offs[hi])], torch.from_numpy(offs[lo:hi + 1] - offs[lo]).to(dev), hi - lo)
             for lo, hi in zip(cuts, cuts[1:])] if K > 1 else None

    def step():
        nonlocal cols, items
        if K > 1:
            r = dec.decode_device_many(parts, out=cols, items=bool(a.ingest_items),
                                       item_cap=2 * n if a.ingest_items else None)
        elif a.ingest_items:
            r = dec.decode_device(buf, off, n, out=cols, items=True, item_cap=2 * n)
        else:
            r = dec.decode_device(buf, off, n, out=cols)
        cols, rej = r[0], r[1]
        if a.ingest_items:
            items = (r[2], r[3])
        assert rej == 0 and cols.n == n

    wall, ev_ms = _timed(step, a.steps, a.warmup, stream)
    per_batch_ms = None
    if K > 1:  # the same batches one decode call each (what the multi-batch call replaces), warm
        from zipkin_amd.columns import DeviceColumns as _DC

        pool = _DC(n, device=f"cuda:{dev.index}")
        ts = []
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            at = 0
            for pb, po, pn in parts:
                if a.ingest_items:
                    dec.decode_device(pb, po, pn, out=pool.slice(at, at + pn), items=True, item_cap=2 * pn)
                else:
                    dec.decode_device(pb, po, pn, out=pool.slice(at, at + pn))
                at += pn
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        per_batch_ms = sorted(ts)[1]
        del pool
    # CPU baseline: the host decoder (zk_ingest_spans, its own pool of up to 16 threads) on the
    # ~200k-fragment set, warm: one untimed decode starts the pool and fills the dictionary, then the
    # median of 5 timed decodes
    hd = SpanDecoder()
    hcols, _ = hd.decode(blobs)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        hd.decode(blobs)
        ts.append(time.perf_counter() - t0)
    cpu_s = sorted(ts)[2]
    cpu_threads = max(1, min(16, os.cpu_count() or 1, m // 2048))  # zk_ingest.cpp kIngestThreads / MinPerThread
    # parity leg: the first and the last replica of the device's decoded columns == the host decoder
    # (zk_ingest_spans) on the same fragments, service ids compared by name (each decoder numbers its
    # own dictionary in the order it meets the names)
    dnames, hnames = dec.service_names(), hd.service_names()
    bad = []
    all_host = cols.to_host(n)
    for rep in sorted({0, reps - 1}):
        got = all_host.take(slice(rep * m, (rep + 1) * m))
        for k in ("trace_id", "span_id", "parent_id", "first_ts", "last_ts", "flags"):
            if not np.array_equal(getattr(got, k), getattr(hcols, k)):
                bad.append(f"{k}@{rep}")
        if [dnames[i] for i in got.service_id.tolist()] != [hnames[i] for i in hcols.service_id.tolist()]:
            bad.append(f"service@{rep}")
    if bad:
        raise RuntimeError(f"ingest: device decode differs from the host decoder: {bad}")
    parity = {"result": "exact", "fragments": 2 * m if reps > 1 else m,
              "checked": "all 7 columns of the first and last replica (service ids by name) == the host decoder "
                         "zk_ingest_spans on the same bytes"}
    if a.ingest_items:
        _, _, (hks, hkh), (has_, hah) = hd.decode(blobs, items=True)
        hid = {nm: i for i, nm in enumerate(hnames)}
        d2h = np.array([hid.get(nm, -1) for nm in dnames], np.int64)  # device id -> host id (by name)
        for (ds, dh), hs, hh, kind in ((items[0], hks, hkh, "kv"), (items[1], has_, hah, "annotation")):
            got_s, got_h = d2h[ds.cpu().numpy().astype(np.int64)], dh.cpu().numpy()
            want_s, want_h = np.tile(hs.astype(np.int64), reps), np.tile(hh.view(np.int64), reps)
            go, wo = np.lexsort((got_h, got_s)), np.lexsort((want_h, want_s))
            if not (np.array_equal(got_s[go], want_s[wo]) and np.array_equal(got_h[go], want_h[wo])):
                raise RuntimeError(f"ingest: device {kind} items differ from the host decoder's")
        parity["items"] = ("key-value and annotation items of the whole batch == the host decoder's items of the "
                           "set x replicas, as multisets of (service name, hash)")
    value = n * a.steps / wall
    algo = in_bytes + n * BYTES_PER_RECORD
    achieved = algo / (ev_ms / a.steps * 1e-3) / 1e9
    print(json.dumps({
        "metric": "stored span fragments/sec decoded into columns (Snappy + thrift, on device)"
                  + (" with the span indexer's items" if a.ingest_items else ""),
        "value": value, "unit": "fragments/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": wall * 1e3 / a.steps, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u8", "data": "synthetic (tracegen records as thrift Spans, Snappy-compressed, replicated)",
        "config": {"workload": f"ingest: {n:.3g} fragments per step, {in_bytes / n:.1f} B each compressed"
                               + (f", as {K} stored batches decoded by one multi-batch call" if K > 1 else ""),
                   "fragments": n, "input_bytes": in_bytes, "batches": K},
        "roofline": {"bound": "hbm", "kernel": "whole decode (5 kernels + 2 scans)", "achieved": achieved,
                     "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS,
                     "algorithmic_bytes_per_step": algo},
        "cpu_baseline": {"value": m / cpu_s, "unit": "fragments/s", "cores": cpu_threads, "kind": "port",
                         "cpu": cpu_model(),
                         "sample": f"{m} fragments through the host decoder (zk_ingest_spans, {cpu_threads} threads, "
                                   f"warm pool and dictionary), median of 5: {cpu_s * 1e3:.1f} ms"},
        "parity": parity,
        "detail": {"event_ms_per_step": ev_ms / a.steps, "services": dec.num_services,
                   **({"one_call_per_batch_ms": per_batch_ms} if per_batch_ms is not None else {})},
    }), flush=True)


def bench_c5(a):
    """BASELINE configs[4] (one GPU): per-service HyperLogLog of distinct traceIds + duration
    histogram (p50/p99) over 1e9 TraceGen spans (the stated "over 1B spans"), fed by K1 in
    sketch-only mode (40 B/record: parentId is not read) + service partition + LDS sketch units.
    Parity and the CPU baseline: oracle/zk_rt_port.c on the first 1e8 records (whole traces)."""
    import torch

    from zipkin_amd import DepsContext, DeviceColumns, tracegen_params
    import numpy as np

    from zipkin_amd.realtime import RtSketch

    # N > 1 (configs[4]: "RCCL max/merge across 8 GPUs"): ONE global set of a.records spans sharded by
    # mix64(traceId) % N like C3; every step merges the ranks' sketches with zk_rt_allreduce (HLL
    # registers by MAX, histogram bins by SUM) through the library's own communicator
    world, rank, local, dist = init_dist()
    dev = torch.device("cuda", local)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    S = a.services
    ctx = DepsContext(S, device=local, stream=stream.cuda_stream, timing=True)
    rt = RtSketch(S, device=local, stream=stream.cuda_stream)
    rt.bind(ctx, only=True)
    p = tracegen_params(a.seed, int(a.records / 15) + 1000, target_records=a.records, max_depth=a.max_depth,
                        num_services=S, rank=rank, world=world, global_ids=world > 1)
    cap = a.records if world == 1 else int(a.records / world * 1.02) + 1_000_000
    cols = DeviceColumns(cap, device=f"cuda:{local}", packed=a.layout == "packed")
    n, ntr = ctx.tracegen_device(p, cols)
    total = n
    if dist is not None:
        tt = torch.tensor([n], dtype=torch.int64, device=dev)
        dist.all_reduce(tt)
        total = int(tt.item())
    comms = (zk_comms(dist, rank, world, local, 2 if a.pipeline != 0 else 1)
             if dist is not None and a.comm == "zk" else None)

    def merge(r, i):
        if dist is None:
            return
        if comms is not None:
            comms[i].allreduce_rt(r)  # zk_rt_allreduce on the sketch's stream
        else:
            from zipkin_amd.shards import merge_rt
            merge_rt(r, device=local)

    def step_serial():
        ctx.reset()
        rt.reset()
        ctx.accumulate(cols, clustered=True, verify=False, n=n)
        merge(rt, 0)

    # K1 alone: a few serial steps before the timed run (untimed)
    step_serial()
    torch.cuda.synchronize()
    tmi = ctx.timing()
    for _ in range(3):
        step_serial()
    tmj = ctx.timing()
    k1_isolated_ms = (tmj["join_ms_total"] - tmi["join_ms_total"]) / (tmj["join_calls"] - tmi["join_calls"])

    step = step_serial
    if a.pipeline != 0:
        # two context/sketch/stream sets: batch k's K1 overlaps batch k-1's partition + sketch
        stream2 = torch.cuda.Stream(device=dev)
        ctx2 = DepsContext(S, device=local, stream=stream2.cuda_stream, timing=False)
        rt2 = RtSketch(S, device=local, stream=stream2.cuda_stream)
        rt2.bind(ctx2, only=True)
        sets = [(ctx, rt, stream), (ctx2, rt2, stream2)]
        k = [0]

        def step():  # noqa: F811
            i = k[0] % 2
            c, r, s = sets[i]
            k[0] += 1
            torch.cuda.set_stream(s)
            c.reset()
            r.reset()
            c.accumulate(cols, clustered=True, verify=False, n=n)
            merge(r, i)

    tm0 = ctx.timing()
    if dist is not None:
        torch.cuda.synchronize()
        dist.barrier()
    wall, ev_ms = _timed(step, a.steps, max(2, a.warmup), stream, [sets[1][2]] if a.pipeline != 0 else ())
    if dist is not None:
        dist.barrier()
        t = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    torch.cuda.set_stream(stream)
    tm1 = ctx.timing()
    calls = tm1["join_calls"] - tm0["join_calls"]
    join_ms = (tm1["join_ms_total"] - tm0["join_ms_total"]) / max(1, calls)
    if a.pipeline != 0:
        # both sets sketched the same batch: registers and bins must agree exactly
        (ra, ha), (rb, hb) = rt.read(), rt2.read()
        if not (np.array_equal(ra, rb) and np.array_equal(ha, hb)):
            raise RuntimeError("pipelined C5 step: the two sketch sets differ")
        rt2.close()
        ctx2.close()
    # the query path of every service at once: distinct estimates + p50/p99 bins (one device pass
    # and one copy each, zk_rt_distinct_traces / zk_rt_quantiles_all); the first call sets up its
    # buffers, the median of 5 warm calls is the steady state
    qt = []
    for _ in range(6):
        t0 = time.perf_counter()
        est = rt.distinct_traces()
        qlo, qhi, qcnt = rt.quantiles_all((0.5, 0.99))
        qt.append((time.perf_counter() - t0) * 1e3)
    query_first_ms, query_ms = qt[0], sorted(qt[1:])[2]
    achieved = n * 40 / (k1_isolated_ms * 1e-3) / 1e9  # K1 alone (serial launches), as in the c2 line
    cpu = parity = None
    if dist is not None:
        # every rank holds the merged sketch: registers and bins must agree across ranks
        import hashlib

        regs, hist = rt.read()
        dg = hashlib.sha256(regs.tobytes() + hist.tobytes()).hexdigest()
        dgs = [None] * world
        dist.all_gather_object(dgs, dg)
        if len(set(dgs)) != 1:
            raise RuntimeError(f"C5 at N = {world}: the ranks' merged sketches differ")
        parity = {"ranks_agree": True, "sha256": dg,
                  "checked": "HLL registers + histogram bins of every service identical on every rank after "
                             "the all-reduce"}
    elif a.cpu_sample > 0:
        cpu, parity = c5_parity_and_baseline(cols, min(a.cpu_sample, n), S, stream, a.cpu_threads or usable_cpus())
    for cm in comms or ():
        cm.close()
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    print(json.dumps({
        "metric": f"spans/sec into per-service HLL distinct traceIds + duration p50/p99 (BASELINE configs[4], {world} GPU)",
        "value": total * a.steps / wall, "unit": "spans/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": wall * 1e3 / a.steps, "higher_is_better": True,
        "scaling": "weak" if world == 1 else "strong", "vs_baseline": None,
        "dtype": "u64", "data": "synthetic (zipkin-tracegen-shaped, generated on device)",
        "config": {"workload": f"C5: {n:.3g} span records (BASELINE configs[4]: over 1B spans), {S} services, "
                               "HLL p=14 + log-linear histogram m=7 (t-digest p50/p99 built from it)",
                   "records": total, "records_per_gpu": n, "traces_per_gpu": ntr, "services": S,
                   "collective": (None if world == 1 else "zk_rt_allreduce (libzkagg's RCCL communicator)"
                                  if comms is not None else "torch.distributed (zipkin_amd/shards.merge_rt)"),
                   "step": "reset + K1 (merge, isValid, serviceName, duration; sketch items) + partition + sketch"
                           + (" (two sets: batch k's K1 overlaps batch k-1's partition + sketch)" if a.pipeline else "")},
        "roofline": {"bound": "hbm", "kernel": "k_span_join_stream<..., kModeEmit>", "achieved": achieved,
                     "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS,
                     "algorithmic_bytes_per_launch": n * 40, "avg_launch_ms": k1_isolated_ms, "launches": 3,
                     "timing": "HIP events on the ctx stream around each K1 launch of serial (non-overlapped) steps"},
        "cpu_baseline": cpu,
        "parity": parity,
        "detail": {"event_ms_per_step": ev_ms / a.steps, "query_ms_all_services": query_ms,
                   "query_first_ms_all_services": query_first_ms,
                   "pipelined_k1_event_ms": join_ms,
                   "median_distinct_estimate": float(sorted(est)[S // 2]),
                   "p50_p99_bins_service0": [(int(qlo[0][i]), int(qhi[0][i])) for i in range(2)]},
    }), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def bench_c1(a):
    """BASELINE configs[0], "C1": the reference's own CPU-runnable case -- the dependency job on 10k
    zipkin-tracegen traces (maxDepth 7, 20 services, seed 1; ~0.3M records). The GPU path runs it
    from HBM (reset + accumulate + finalize per step, like C2); the CPU baseline is the port on all
    usable cores, median of 10 runs, as BASELINE.md asks; both are checked against the oracle."""
    import numpy as np
    import torch

    from oracle import oracle
    from zipkin_amd import DepsContext, DeviceColumns, tracegen_host

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    S, T = 20, 10_000
    host = tracegen_host(1, T, max_depth=7, num_services=S)
    n = len(host)
    cols = DeviceColumns.from_host(host, device="cuda:0")
    # no per-phase events: C1 reports the step only, and at 0.15 ms per step the library's eight
    # event records per step are a visible part of it
    ctx = DepsContext(S, device=0, stream=stream.cuda_stream, timing=os.environ.get("ZK_C1_TIMING") == "1")
    out = {k: torch.empty(S * S, dtype=dt, device=dev) for k, dt in
           (("m0", torch.int64), ("m1", torch.float64), ("m2", torch.float64), ("m3", torch.float64),
            ("m4", torch.float64), ("present", torch.uint8))}

    def step():
        ctx.reset()
        ctx.accumulate(cols, clustered=True, verify=False)
        ctx.finalize(out_device=out)

    wall, ev_ms = _timed(step, a.steps, a.warmup, stream)
    got = ctx.finalize()
    st = ctx.stats()
    ref = oracle.aggregate(host, S)
    m0, ms = ref.dense()
    if not (np.array_equal(got.m0, m0) and all(np.array_equal(x, y) for x, y in zip((got.m1, got.m2, got.m3, got.m4), ms))
            and all(st[k] == v for k, v in ref.stats.items() if k != "spilled_traces")):
        raise RuntimeError("C1: GPU result differs from the oracle")
    threads = a.cpu_threads or usable_cpus()
    times = []
    for _ in range(11):  # one warm-up + 10 timed
        rp = oracle.aggregate_port(host, S, threads=threads, clustered=True)
        times.append(rp.seconds)
    cpu_s = float(np.median(times[1:]))
    if not (np.array_equal(rp.cells, ref.cells) and rp.stats == ref.stats):
        raise RuntimeError("C1: CPU port differs from the oracle")
    ctx.close()
    print(json.dumps({
        "metric": "spans/sec into DependencyLinks (BASELINE configs[0]: 10k tracegen traces, 20 services)",
        "value": n * a.steps / wall, "unit": "spans/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": wall * 1e3 / a.steps, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u64", "data": "synthetic (zipkin-tracegen-shaped, seed 1)",
        "config": {"workload": "C1: 10k tracegen traces, maxDepth 7, 20 services", "records": n, "traces": T,
                   "services": S, "step": "reset + span_join + spill + finalize(m0..m4) + status check"},
        "parity": {"result": "exact", "records": n, "links": int(got.present.sum()),
                   "checked": "GPU and CPU port vs oracle/zk_oracle.c: m0..m4 bit-identical + counters"},
        "cpu_baseline": {"value": n / cpu_s, "unit": "spans/s", "cores": threads, "kind": "port", "cpu": cpu_model(),
                         "sample": f"the whole C1 batch ({n} records), oracle/zk_cpu_port.c, median of 10: "
                                   f"{cpu_s * 1e3:.2f} ms"},
        "detail": {"event_ms_per_step": ev_ms / a.steps, "note": "a 14 MB batch: launch- and latency-bound on the GPU"},
    }), flush=True)


def bench_c4(a):
    """BASELINE configs[3] (one GPU slice): getTopKeyValueAnnotations via count-min + top-K over
    binary annotations (service u32, key hash u64 = 12 B/item), Zipf(1.1) keys over 1e6 ids,
    services uniform over 500, generated on device."""
    import torch

    import numpy as np

    from zipkin_amd.kv import KvSketch

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    S, n = a.services, a.items
    g = torch.Generator(device=dev)
    g.manual_seed(4)
    w = 1.0 / torch.arange(1, 1_000_001, dtype=torch.float64, device=dev) ** 1.1
    cdf = torch.cumsum(w, 0)
    cdf /= cdf[-1].clone()
    keys = torch.empty(n, dtype=torch.int64, device=dev)
    svc = torch.randint(0, S, (n,), dtype=torch.int32, device=dev, generator=g)
    M = (1 << 64) - 1

    def s64(c):  # a uint64 constant as the int64 torch multiplies with (two's complement wrap)
        return c - (1 << 64) if c >= 1 << 63 else c

    def shr(x, k):  # logical right shift on int64
        return (x >> k) & ((1 << (64 - k)) - 1)

    chunk = 50_000_000
    for b in range(0, n, chunk):
        e = min(n, b + chunk)
        r = torch.searchsorted(cdf, torch.rand(e - b, dtype=torch.float64, device=dev, generator=g), right=True)
        z = r.to(torch.int64) + 0x5EED
        z = (z ^ shr(z, 30)) * s64(0xBF58476D1CE4E5B9)
        z = (z ^ shr(z, 27)) * s64(0x94D049BB133111EB)
        keys[b:e] = z ^ shr(z, 31)
    del M
    kv = KvSketch(S, stream=stream.cuda_stream, seed=4, timing=True)

    def step():
        kv.reset()
        kv.accumulate(svc, keys)

    others = ()
    if a.pipeline != 0:
        # two sketch/stream sets: batch k's partition overlaps batch k-1's sketch + candidates
        stream2 = torch.cuda.Stream(device=dev)
        kv2 = KvSketch(S, stream=stream2.cuda_stream, seed=4)
        sets = [(kv, stream), (kv2, stream2)]
        others = (stream2,)
        k = [0]

        def step():  # noqa: F811
            c, s = sets[k[0] % 2]
            k[0] += 1
            torch.cuda.set_stream(s)
            c.reset()
            c.accumulate(svc, keys)

    wall, ev_ms = _timed(step, a.steps, max(2, a.warmup), stream, others)
    torch.cuda.set_stream(stream)
    t0 = time.perf_counter()
    kk, est, cnt = kv.topk_all(10)
    query_first_ms = (time.perf_counter() - t0) * 1e3
    qt = []
    for _ in range(5):  # a query server's steady state: the first call pays one-time HIP setup
        t0 = time.perf_counter()
        kv.topk_all(10)
        qt.append((time.perf_counter() - t0) * 1e3)
    query_ms = sorted(qt)[2]
    if a.pipeline != 0:
        kk2, est2, cnt2 = kv2.topk_all(10)
        if not (np.array_equal(kk, kk2) and np.array_equal(est, est2) and np.array_equal(cnt, cnt2)):
            raise RuntimeError("pipelined C4 step: the two sketch sets differ")
        kv2.close()
    # per-phase device time of isolated (serial) steps, HIP events inside zk_kv_accumulate
    ph = []
    for _ in range(3):
        kv.reset()
        kv.accumulate(svc, keys)
        ph.append(kv.phase_ms())
    phase = {k: float(np.median([p[k] for p in ph])) for k in ph[0]}
    # algorithmic bytes per item: the partition reads the item (12 B) and writes its key in service
    # order (8 B); the sketch and candidate passes each read the sorted key (8 B)
    per_item = {"partition": 20, "sketch": 8, "candidates": 8}
    kernels = {k: {"ms": phase[k], "bytes": n * b, "achieved_GBs": n * b / (phase[k] * 1e-3) / 1e9,
                   "frac": n * b / (phase[k] * 1e-3) / 1e9 / PEAK_HBM_GBS} for k, b in per_item.items()}
    value = n * a.steps / wall
    achieved = n * 12 / (ev_ms / a.steps * 1e-3) / 1e9  # HIP events on the step's stream
    cpu = parity = None
    if a.cpu_sample > 0:
        cpu, parity = c4_parity_and_baseline(svc, keys, min(a.cpu_sample, n), S, kv, stream,
                                             a.cpu_threads or usable_cpus())
    print(json.dumps({
        "metric": "binary annotations/sec into per-service count-min + top-K (BASELINE configs[3], 1 GPU)",
        "value": value, "unit": "annotations/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": wall * 1e3 / a.steps, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "u32", "data": "synthetic (Zipf(1.1) keys over 1e6 ids, 500 services, generated on device)",
        "config": {"workload": f"C4: {n:.3g} binary annotations per step, count-min 4 x {kv.width} per service, K=64 kept",
                   "items": n, "services": S,
                   "count_min": f"depth {kv.depth} x width {kv.width} per service = {kv.depth * kv.width * S / 2**20:.2f} Mi "
                                "u32 counters, the memory of SURVEY 8d's d=4, w=2^20; per-service error e/w x N_s "
                                f"= {2.718281828 / kv.width / S:.3g} N with N_s = N/S, the same absolute bound as one "
                                "global 4 x 2^20 sketch (e/2^20 N = 2.59e-6 N), delta = e^-4",
                   "step": "reset + partition + sketch + candidates + merge"
                           + (" (two sets: batch k overlaps batch k-1)" if a.pipeline else "")},
        "roofline": {"bound": "hbm", "kernel": "whole step (partition + sketch + candidates + merge)",
                     "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": achieved / PEAK_HBM_GBS,
                     "algorithmic_bytes_per_step": n * 12},
        "kernels": kernels,
        "cpu_baseline": cpu,
        "parity": parity,
        "detail": {"event_ms_per_step": ev_ms / a.steps, "topk_query_ms": query_ms, "topk_query_first_ms": query_first_ms,
                   "service0_top3": [(int(k), int(e)) for k, e in zip(kk[0][:3], est[0][:3])]},
    }), flush=True)


def c5_parity_and_baseline(cols, sample, S, stream, threads):
    """C5's parity leg and CPU baseline on the first `sample` records (whole traces) of the timed
    batch: a fresh device sketch fed by K1's emit mode over that prefix against oracle/zk_rt_port.c
    (the C restatement of oracle/realtime.py, pinned to it by tests/test_realtime.py: Span.mergeSpan
    / isValid / serviceName / duration, HyperLogLog registers, log-linear histogram) -- every
    register, bin, drop count and estimate identical, else the bench fails. The port's own time on
    the prefix (median of 3, all usable cores) is the baseline (kind "port")."""
    import numpy as np

    from oracle.realtime import rt_port
    from zipkin_amd import DepsContext
    from zipkin_amd.realtime import RtSketch

    host = cols.to_host(sample + 100_000)
    cut = min(sample, len(host))
    while 0 < cut < len(host) and host.trace_id[cut] == host.trace_id[cut - 1]:
        cut -= 1
    part = host.take(slice(0, cut))
    with DepsContext(S, stream=stream.cuda_stream) as ctx, RtSketch(S, stream=stream.cuda_stream) as rt:
        rt.bind(ctx, only=True)
        ctx.accumulate(cols, clustered=True, verify=False, n=cut)
        gr, gh = rt.read()
        gd = rt.distinct_traces()
        gdrop = rt.dropped()
        rt.unbind()
    times = []
    for _ in range(3):
        o = rt_port(part, S, p=rt.p, m=rt.m, seed=0, threads=threads)
        times.append(o.seconds)
    secs = sorted(times)[1]
    bad = [k for k, ok in (("registers", np.array_equal(gr, o.regs)), ("histogram", np.array_equal(gh, o.hist)),
                           ("estimates", np.array_equal(gd, o.distinct())),
                           ("dropped", gdrop == (o.dropped_service, o.dropped_duration))) if not ok]
    if bad:
        raise RuntimeError(f"C5 parity failure on the {cut}-record prefix: {bad}")
    cpu = {"value": cut / secs, "unit": "spans/s", "cores": threads, "kind": "port", "cpu": cpu_model(),
           "sample": f"first {cut} records (whole traces) of the benchmark batch; oracle/zk_rt_port.c (merge, "
                     f"isValid, serviceName, duration, HLL p={rt.p}, histogram m={rt.m}), {threads} threads, "
                     f"median of 3: {secs:.3f} s"}
    parity = {"result": "exact", "records": cut,
              "checked": "every HLL register, histogram bin, drop count and distinct estimate of all services, "
                         "fresh device sketch (K1 emit mode) of the prefix vs oracle/zk_rt_port.c "
                         "(== oracle/realtime.py, tests/test_realtime.py)"}
    return cpu, parity


def c4_parity_and_baseline(svc, keys, sample, S, kv_geom, stream, threads):
    """C4's parity leg and CPU baseline on the first `sample` items of the timed batch: a fresh
    device sketch of that prefix against oracle/zk_kv_port.c (the C restatement of oracle/kv.py,
    pinned to it by tests/test_kv.py): every service's full candidate list (keys and estimates, in
    order) and the per-service totals must be identical, else the bench fails. The port's own time
    on the prefix (median of 3, all usable cores) is the baseline (kind "port")."""
    import numpy as np

    from oracle.kv import kv_port
    from zipkin_amd.kv import KvSketch

    hs = svc[:sample].cpu().numpy().view(np.uint32)
    hk = keys[:sample].cpu().numpy().view(np.uint64)
    cand = kv_geom.candidates
    with KvSketch(S, stream=stream.cuda_stream, seed=4) as g:
        g.accumulate(svc[:sample], keys[:sample])
        gk, ge, gc = g.topk_all(cand)
        gt = g.totals()
    times = []
    for _ in range(3):
        p = kv_port(hs, hk, S, kv_geom.width, kv_geom.depth, cand, seed=4, threads=threads)
        times.append(p.seconds)
    pk, pe, pc = p.topk_all(cand)
    bad = [k for k, x, y in (("keys", gk, pk), ("estimates", ge, pe), ("counts", gc, pc), ("totals", gt, p.totals))
           if not np.array_equal(x, y)]
    if bad:
        raise RuntimeError(f"C4 parity failure on the {sample}-item prefix: {bad}")
    t = sorted(times)[1]
    cpu = {"value": sample / t, "unit": "annotations/s", "cores": threads, "kind": "port", "cpu": cpu_model(),
           "sample": f"first {sample} items of the benchmark batch; oracle/zk_kv_port.c (count-min + top-{cand} per "
                     f"service, {threads} threads), median of 3: {t:.3f} s"}
    parity = {"result": "exact", "items": sample,
              "checked": f"all {S} services' top-{cand} candidate lists (keys, estimates, order) and totals, fresh "
                         "device sketch of the prefix vs oracle/zk_kv_port.c (== oracle/kv.py, tests/test_kv.py)"}
    return cpu, parity


if __name__ == "__main__":
    main()
