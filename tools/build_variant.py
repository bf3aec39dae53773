#!/usr/bin/env python3
"""Build an A/B variant of libzkagg: the sources of a git revision (default: the working tree) with
optional -D defines, into zipkin_amd/libzkagg_<name>.so (run with ZKAGG_LIB=... or tools/ab.sh).

  python tools/build_variant.py NAME [--rev REV] [-D DEFINE ...] [--flag=COMPILER_FLAG ...]
"""
import argparse
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
from zipkin_amd import build as zb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--rev", default=None)
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--flag", action="append", default=[], help="extra compiler flag (e.g. --flag=-mllvm=-x)")
    a = ap.parse_args()
    tmp = Path(tempfile.mkdtemp(prefix="zkvar_"))
    try:
        if a.rev:
            for sub in ("zipkin_amd/csrc", "include"):
                (tmp / sub).mkdir(parents=True)
                files = subprocess.run(["git", "-C", str(ROOT), "ls-tree", "--name-only", f"{a.rev}:{sub}"],
                                       check=True, capture_output=True, text=True).stdout.split()
                for f in files:
                    data = subprocess.run(["git", "-C", str(ROOT), "show", f"{a.rev}:{sub}/{f}"], check=True,
                                          capture_output=True).stdout
                    (tmp / sub / f).write_bytes(data)
        else:
            shutil.copytree(ROOT / "zipkin_amd" / "csrc", tmp / "zipkin_amd" / "csrc")
            shutil.copytree(ROOT / "include", tmp / "include")
        csrc = tmp / "zipkin_amd" / "csrc"
        srcs = [s for s in zb.SOURCES if (csrc / s).exists()]
        flags = [f"--offload-arch={zb.ARCH}", "-O3", "-fPIC", "-std=c++17", "-Wno-unused-result",
                 "-Wno-unused-value", f"-I{tmp / 'include'}"] + [f"-D{d}" for d in a.D] + [
                     x for f in a.flag for x in (f.split("=", 1) if f.startswith("-mllvm=") else [f])]

        def cc(src):
            obj = tmp / (src + ".o")
            subprocess.run([zb._hipcc(), *flags, "-c", str(csrc / src), "-o", str(obj)], check=True)
            return obj

        with ThreadPoolExecutor(max_workers=8) as ex:
            objs = list(ex.map(cc, srcs))
        out = ROOT / "zipkin_amd" / f"libzkagg_{a.name}.so"
        subprocess.run([zb._hipcc(), f"--offload-arch={zb.ARCH}", "-shared", "-fPIC", *map(str, objs), "-L/opt/rocm/lib",
                        "-lrocprofiler-sdk-roctx", "-ldl", "-Wl,-rpath,/opt/rocm/lib", "-o", str(out)], check=True)
        print(out)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
