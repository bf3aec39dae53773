"""Diagnostic: shuffled vs clustered C2-shaped batches at several sizes (library clustering pass vs a
torch stable sort by traceId feeding the clustered path)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from zipkin_amd import DepsContext, DeviceColumns, tracegen_params  # noqa: E402

COLS = ("trace_id", "span_id", "parent_id", "first_ts", "last_ts", "service_id", "flags")


def run(ctx_args, cols, n, clustered, verify=False):
    with DepsContext(500, device=0, **ctx_args) as c:
        c.accumulate(cols, clustered=clustered, verify=verify, n=n)
        try:
            out = c.finalize()
            err = None
        except Exception as e:  # noqa: BLE001
            out, err = None, str(e)
        return out, c.stats(), err


def main():
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    for N in [int(x) for x in sys.argv[1:]] or [2_000_000, 20_000_000, 100_000_000]:
        with DepsContext(500, device=0) as g:
            p = tracegen_params(2, int(N / 15) + 1000, target_records=N, max_depth=6, num_services=500)
            cols = DeviceColumns(N, device="cuda:0")
            n, ntr = g.tracegen_device(p, cols)
        torch.cuda.synchronize()
        gen = torch.Generator(device=dev)
        gen.manual_seed(7)
        perm = torch.randperm(n, device=dev, generator=gen)
        sc = DeviceColumns(n, device="cuda:0")
        for k in COLS:
            torch.index_select(getattr(cols, k)[:n], 0, perm, out=getattr(sc, k))
        # torch clustering of the shuffled batch: stable sort by the unsigned traceId
        key = sc.trace_id ^ (-(2**63))
        _, order = torch.sort(key, stable=True)
        tc = DeviceColumns(n, device="cuda:0")
        for k in COLS:
            torch.index_select(getattr(sc, k), 0, order, out=getattr(tc, k))
        torch.cuda.synchronize()
        t0 = time.time()
        r0, s0, e0 = run({}, cols, n, True, verify=True)
        r1, s1, e1 = run({}, sc, n, False, verify=True)
        r2, s2, e2 = run({}, tc, n, True, verify=True)
        diff1 = {k: (s0[k], s1[k]) for k in s0 if s0[k] != s1[k]}
        diff2 = {k: (s0[k], s2[k]) for k in s0 if s0[k] != s2[k]}
        print(f"N={n} traces={ntr} errs={e0},{e1},{e2}", flush=True)
        print(f"  lib-clustered vs orig: {diff1}", flush=True)
        print(f"  torch-clustered vs orig: {diff2}", flush=True)
        if r0 is not None and r1 is not None:
            print(f"  m0 equal lib: {bool((r0.m0 == r1.m0).all())}  torch: {bool((r0.m0 == r2.m0).all()) if r2 else None}",
                  flush=True)
        print(f"  took {time.time() - t0:.1f}s", flush=True)
        del cols, sc, tc, perm, order, key
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
