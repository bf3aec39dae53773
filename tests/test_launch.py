"""Launch hygiene (zipkin_amd/csrc/zk_launch.h), checked on the CPU against the built library.

Round 2 dispatched k_part_scatter_lines at S = 1024 with a 163,968-byte group segment -- more than
the 160 KiB of a CU, which the HIP runtime does not refuse -- and it faulted. Every launch now goes
through launch_checked, which reads the kernel's static LDS from its code object and refuses a
launch that does not fit; planners with a fallback ask the same rule first. These tests read every
kernel's static LDS from the gfx950 code objects inside libzkagg.so (no GPU needed) and check:
no kernel's static LDS exceeds a CU; the partition planner picks the line scatter only where it
fits, else the item scatter, at every S boundary; the other dynamic-LDS launches fit at the largest
configuration the library accepts; and no source launches a kernel outside launch_checked."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

from zipkin_amd import _abi

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "zipkin_amd" / "csrc"
LLVM = Path("/opt/rocm/lib/llvm/bin")
LDS_PER_CU = 160 * 1024


def _static_lds(tmp_path_factory) -> dict:
    """{kernel symbol: .group_segment_fixed_size} over every gfx950 code object in the library."""
    lib = Path(_abi.lib()._name)
    d = tmp_path_factory.mktemp("codeobj")
    fat = d / "fatbin.bin"
    subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(lib), str(d / "x.so")],
                   check=True)
    blob = fat.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), blob)] + [len(blob)]
    out = {}
    for i, (a, b) in enumerate(zip(starts, starts[1:])):
        part = d / f"b{i}.bin"
        part.write_bytes(blob[a:b])
        hsaco = d / f"b{i}.hsaco"
        r = subprocess.run([str(LLVM / "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={hsaco}"],
                           capture_output=True)
        if r.returncode != 0 or not hsaco.exists() or hsaco.stat().st_size == 0:
            continue
        notes = subprocess.run([str(LLVM / "llvm-readelf"), "--notes", str(hsaco)], capture_output=True,
                               text=True, check=True).stdout
        size = None
        for line in notes.splitlines():
            m = re.search(r"\.group_segment_fixed_size:\s*(\d+)", line)
            if m:
                size = int(m.group(1))
            m = re.search(r"^\s*\.name:\s*(\S+)", line)
            if m and size is not None:
                out[m.group(1)] = size
                size = None
    return out


@pytest.fixture(scope="module")
def lds(tmp_path_factory):
    if not (LLVM / "clang-offload-bundler").exists():
        pytest.skip("ROCm LLVM tools not present")
    got = _static_lds(tmp_path_factory)
    assert len(got) >= 30, f"found only {len(got)} kernels in the code objects"
    return got


def _one(lds, needle):
    hits = {k: v for k, v in lds.items() if needle in k}
    assert hits, f"no kernel matching {needle}"
    return max(hits.values())


def test_every_kernel_static_lds_fits_a_cu(lds):
    over = {k: v for k, v in lds.items() if v > LDS_PER_CU}
    assert not over


@pytest.mark.parametrize("S", [1, 500, 1021, 1022, 1023, 1024, 2048, 4096])
def test_partition_planner_never_dispatches_over_budget(lds, S):
    L = _abi.lib()
    f = L.zk_internal_partition_choice
    f.restype = C.c_int
    f.argtypes = [C.c_uint32, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64)]
    st_lines = _one(lds, "k_part_scatter_lines")
    st_items = _one(lds, "k_part_scatter")
    dyn = C.c_uint64()
    choice = f(S, st_lines, st_items, C.byref(dyn))
    assert choice in (-1, 0, 1)
    if choice == 1:  # line scatter: static + the [S][8] u64 carry
        assert dyn.value == S * 64 and st_lines + dyn.value <= LDS_PER_CU
    elif choice == 0:  # item scatter: static + S u32 cursors
        assert dyn.value == S * 4 and st_items + dyn.value <= LDS_PER_CU
        # the fallback is taken only where the line scatter does not fit
        assert S > 1024 or st_lines + S * 64 > LDS_PER_CU
    else:
        assert st_items + S * 4 > LDS_PER_CU
    if S == 1024:  # round 2's fault: the line scatter needs 163,968 B there
        assert choice != 1


@pytest.mark.parametrize("S", [1, 23, 500, 724, 1024, 1448, 4096])
def test_reduce_scatter_lds_fits(lds, S):
    f = _abi.lib().zk_internal_dyn_lds
    f.restype = C.c_uint64
    f.argtypes = [C.c_uint32, C.c_uint32]
    dyn = f(0, S)
    assert _one(lds, "k_link_scatter") + dyn <= LDS_PER_CU


def test_sketch_launches_fit_at_their_largest_configuration(lds):
    f = _abi.lib().zk_internal_dyn_lds
    f.restype = C.c_uint64
    f.argtypes = [C.c_uint32, C.c_uint32]
    for k in ("k_kv_sketch", "k_kv_candidates", "k_kv_merge"):
        assert _one(lds, k) + f(1, 0) <= LDS_PER_CU, k
    assert _one(lds, "k_rt_sketch") + f(2, 0) <= LDS_PER_CU


def test_no_launch_outside_launch_checked():
    raw = []
    for p in sorted(CSRC.iterdir()):
        if p.suffix not in (".hip", ".cpp", ".h") or p.name == "zk_launch.h":
            continue
        for i, line in enumerate(p.read_text().splitlines(), 1):
            code = line.split("//")[0]
            if re.search(r"hipLaunchKernelGGL|<<<|hipLaunchKernel\(|hipLaunchCooperativeKernel", code):
                raw.append(f"{p.name}:{i}")
    assert not raw, f"kernel launches outside launch_checked: {raw}"
