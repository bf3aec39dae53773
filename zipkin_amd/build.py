"""Build libzkagg.so in-tree with hipcc for gfx950 (no JIT cache, so the .so travels with the repo)."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
SOURCES = [
    "zk_join.hip",
    "zk_reduce.hip",
    "zk_finalize.hip",
    "zk_tracegen.hip",
    "zk_api.cpp",
    "zk_partition.hip",
    "zk_kv.hip",
    "zk_kv_api.cpp",
    "zk_store.cpp",
    "zk_rt.hip",
    "zk_rt_api.cpp",
    "zk_ingest.cpp",
    "zk_ingest_dev.hip",
    "zk_cluster.hip",
    "zk_launch.cpp",
    "zk_exchange.hip",
    "zk_comm.cpp",
    "zk_rl.hip",
]
HEADERS = ["zk_internal.h", "zk_cluster.h", "zk_tracegen.h", "zk_sketch_internal.h", "zk_rt_internal.h", "zk_block.h", "zk_launch.h", "zk_comm.h", "zk_rl_internal.h"]
PUBLIC_HEADERS = ["zkagg.h", "zksketch.h", "zkstore.h", "zkingest.h", "zkcomm.h"]
LIB = PKG / "libzkagg.so"
ARCH = os.environ.get("ZK_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (Path(c).exists() or c == "hipcc"):
            return c
    raise RuntimeError("hipcc not found")


def needs_build() -> bool:
    if not LIB.exists():
        return True
    t = LIB.stat().st_mtime
    deps = [CSRC / s for s in SOURCES + HEADERS] + [ROOT / "include" / h for h in PUBLIC_HEADERS]
    return any(d.stat().st_mtime > t for d in deps)


def _flags() -> list[str]:
    return [f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result", "-Wno-unused-value",
            f"-I{ROOT / 'include'}"]


def build(force: bool = False, verbose: bool = False, variant: str = "", defines=()) -> Path:
    """Compile every source to an object in build/ (in parallel, only what changed), then link.

    variant/defines: a diagnostic build (e.g. "stamps", ["ZK_STAMPS"]) into libzkagg_<variant>.so;
    the product library is always the plain build."""
    lib = PKG / f"libzkagg_{variant}.so" if variant else LIB
    if not variant and not force and not needs_build():
        return LIB
    from concurrent.futures import ThreadPoolExecutor

    objdir = ROOT / "build" / ("zkagg_" + variant if variant else "zkagg")
    objdir.mkdir(parents=True, exist_ok=True)
    hdr_t = max((CSRC / h).stat().st_mtime for h in HEADERS)
    hdr_t = max([hdr_t] + [(ROOT / "include" / h).stat().st_mtime for h in PUBLIC_HEADERS])

    def compile_one(src: str) -> Path:
        obj = objdir / (src + ".o")
        if force or not obj.exists() or obj.stat().st_mtime < max(hdr_t, (CSRC / src).stat().st_mtime):
            cmd = [_hipcc(), *_flags(), *[f"-D{d}" for d in defines], "-c", str(CSRC / src), "-o", str(obj) + ".tmp"]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            subprocess.run(cmd, check=True)
            os.replace(str(obj) + ".tmp", obj)
        return obj

    with ThreadPoolExecutor(max_workers=min(8, len(SOURCES))) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *[str(o) for o in objs], "-L/opt/rocm/lib",
           "-lrocprofiler-sdk-roctx", "-ldl", "-Wl,-rpath,/opt/rocm/lib", "-o", str(lib) + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(str(lib) + ".tmp", lib)
    return lib


if __name__ == "__main__":
    if "--stamps" in sys.argv:
        print(build(verbose=True, variant="stamps", defines=["ZK_STAMPS"]))
    else:
        print(build(force="--force" in sys.argv, verbose=True))
