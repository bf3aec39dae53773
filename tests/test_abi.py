"""The C-ABI library loads and exports every entry point include/zkagg.h declares (no GPU calls)."""
import ctypes as C
import re
from pathlib import Path

import pytest

from tests.conftest import gpu_available
from zipkin_amd import _abi

INCLUDE = Path(__file__).resolve().parent.parent / "include"


def declared_functions():
    names = set()
    for h in sorted(INCLUDE.glob("*.h")):
        text = re.sub(r"/\*.*?\*/", "", h.read_text(), flags=re.S)
        names |= set(re.findall(r"\b(zk_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


def test_header_declares_what_the_binding_binds():
    assert declared_functions() == sorted(_abi.SYMBOLS)


def test_library_exports_every_declared_symbol():
    L = _abi.lib()
    raw = C.CDLL(str(_abi.LIB_PATH))
    for name in declared_functions():
        assert hasattr(raw, name), name
    assert L.zk_abi_version() == 3


def test_status_strings():
    for s in range(0, 12):
        assert _abi.status_str(s) and _abi.status_str(s) != "unknown status"


def test_ctx_create_rejects_bad_config_without_touching_a_device():
    L = _abi.lib()
    cfg = _abi.zk_config()
    h = C.c_void_p()
    cfg.num_services = 0
    assert L.zk_ctx_create(C.byref(cfg), C.byref(h)) == _abi.ZK_ERR_INVALID_ARG
    cfg.num_services = 5000
    assert L.zk_ctx_create(C.byref(cfg), C.byref(h)) == _abi.ZK_ERR_INVALID_ARG
    assert L.zk_ctx_create(None, C.byref(h)) == _abi.ZK_ERR_INVALID_ARG


@pytest.mark.skipif(gpu_available(), reason="checks the no-device path")
def test_no_device_fails_loudly_instead_of_falling_back():
    from zipkin_amd import DepsContext, ZkError

    with pytest.raises(ZkError) as e:
        DepsContext(10)
    assert e.value.status == _abi.ZK_ERR_NO_DEVICE


def test_null_ctx_calls_are_errors():
    L = _abi.lib()
    assert L.zk_deps_reset(None) == _abi.ZK_ERR_INVALID_ARG
    assert L.zk_ctx_destroy(None) == _abi.ZK_ERR_INVALID_ARG
    assert L.zk_deps_accumulate(None, None, 0) == _abi.ZK_ERR_INVALID_ARG
    n, r = C.c_uint64(), C.c_uint64()
    assert L.zk_ingest_dev_spans_multi(None, 0, None, None, None, 0, 0, None, C.byref(n), C.byref(r),
                                       None) == _abi.ZK_ERR_INVALID_ARG


def test_jni_sources_bind_only_declared_entry_points():
    """jvm/src/main/c/zkagg_jni.c (uncompiled here: no JDK) calls only functions include/*.h
    declares, and every ZkNative @native method has a JNI implementation."""
    root = INCLUDE.parent
    c = (root / "jvm" / "src" / "main" / "c" / "zkagg_jni.c").read_text()
    calls = set(re.findall(r"\b(zk_[a-z0-9_]+)\s*\(", re.sub(r"/\*.*?\*/", "", c, flags=re.S)))
    assert calls and calls <= set(declared_functions()), calls - set(declared_functions())
    scala = (root / "jvm" / "src" / "main" / "scala" / "com" / "twitter" / "zipkin" / "gpu" / "ZkNative.scala").read_text()
    natives = set(re.findall(r"@native def (\w+)", scala))
    implemented = set(re.findall(r"JNICALL FN\((\w+)\)", c))
    assert natives == implemented, natives ^ implemented


def test_comm_rejects_bad_arguments_without_a_collective():
    """zkcomm.h: argument checks come before RCCL or a device is touched."""
    L = _abi.lib()
    uid = (C.c_uint8 * 128)()
    h = C.c_void_p()
    assert L.zk_comm_create(uid, 128, 1, 1, 0, C.byref(h)) == _abi.ZK_ERR_INVALID_ARG  # rank >= world
    assert L.zk_comm_create(uid, 64, 0, 1, 0, C.byref(h)) == _abi.ZK_ERR_INVALID_ARG   # short id
    assert L.zk_comm_create(None, 128, 0, 1, 0, C.byref(h)) == _abi.ZK_ERR_INVALID_ARG
    assert L.zk_comm_unique_id(uid, 16) == _abi.ZK_ERR_INVALID_ARG
    assert L.zk_comm_destroy(None) == _abi.ZK_ERR_INVALID_ARG
    assert L.zk_deps_allreduce(None, None, 0) == _abi.ZK_ERR_INVALID_ARG
    if not gpu_available():
        assert L.zk_comm_create(uid, 128, 0, 1, 0, C.byref(h)) == _abi.ZK_ERR_NO_DEVICE
