"""Driver of tools/microbench/wavesort.hip (not product code): the C2 batch (1e8 TraceGen records,
generated on the device by the library) through the sorted-design floor variants, next to K1 on
the same batch. Prints one JSON line. Build: hipcc --offload-arch=gfx950 -O3 -fPIC -shared
tools/microbench/wavesort.hip -o tools/microbench/libwavesort.so"""
import ctypes as C
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from zipkin_amd import DepsContext, DeviceColumns, tracegen_params  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    L = C.CDLL(str(ROOT / "tools" / "microbench" / "libwavesort.so"))
    L.ws_run.argtypes = [C.c_void_p] * 3 + [C.c_uint64, C.c_int, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_float)]
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    with DepsContext(500, device=0, stream=stream.cuda_stream, timing=True) as ctx:
        p = tracegen_params(2, n // 15 + 1000, target_records=n, max_depth=6, num_services=500)
        cols = DeviceColumns(n)
        nrec, _ = ctx.tracegen_device(p, cols)
        ctx.sync()
        for _ in range(2):
            ctx.reset()
            ctx.accumulate(cols, clustered=True, verify=False, n=nrec)
        t0 = ctx.timing()
        for _ in range(5):
            ctx.reset()
            ctx.accumulate(cols, clustered=True, verify=False, n=nrec)
        t1 = ctx.timing()
        k1 = (t1["join_ms_total"] - t0["join_ms_total"]) / (t1["join_calls"] - t0["join_calls"])
    torch.cuda.synchronize()
    grid = 256 * 8  # 8 workgroups of 4 waves per CU
    out = torch.empty(grid * 256, dtype=torch.int64, device="cuda")
    res = {"records": nrec, "k1_ms": k1}
    for mode, name in ((0, "stream_segments"), (1, "bitonic_sort"), (2, "sort_and_binary_search")):
        ms = C.c_float()
        rc = L.ws_run(cols.trace_id.data_ptr(), cols.span_id.data_ptr(), cols.parent_id.data_ptr(), nrec, mode,
                      out.data_ptr(), grid, 10, C.byref(ms))
        if rc:
            raise RuntimeError("kernel launch failed")
        res[name + "_ms"] = ms.value
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
