"""ASan/UBSan CPU build of the host byte parsers, the store and the oracle (tools/sanitize).

zk_ingest.cpp parses untrusted stored bytes (Snappy + TBinaryProtocol); zk_store.cpp and
oracle/zk_oracle.c do pointer-heavy host work. The driver decodes a corpus of real fragments
(richgen spans through the thrift encoder that is byte-exact with the reference's fixtures) and
thousands of mutated batches -- bit flips, truncations, splices, hostile Snappy headers -- and
exercises every store mode; any sanitizer report aborts the run."""
import os
import shutil
import struct
import subprocess
from pathlib import Path

import pytest

from tests import thriftenc as T
from tests.richgen import gen_traces

ROOT = Path(__file__).resolve().parent.parent
BIN = ROOT / "build" / "sanitize" / "fuzz_host"


@pytest.fixture(scope="module")
def fuzz_bin():
    if not shutil.which("g++"):
        pytest.skip("no host C++ compiler")
    subprocess.run(["make", "-s", "-C", str(ROOT / "tools" / "sanitize")], check=True)
    return BIN


def test_parsers_store_and_oracle_are_sanitizer_clean(fuzz_bin, tmp_path):
    spans = gen_traces(71, 60, max_depth=4, anomalies=0.3)
    corpus = tmp_path / "corpus.bin"
    with open(corpus, "wb") as f:
        for i, s in enumerate(spans):
            raw = T.span(s)
            for blob in (raw, T.snappy(raw)) if i % 2 else (raw,):
                f.write(struct.pack("<I", len(blob)) + blob)
        deps = T.dependencies(0, 3600_000_000, [("web", "db", (3, 1.5, 2.0, 0.0, 4.0))])
        f.write(struct.pack("<I", len(deps)) + deps)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(fuzz_bin), str(corpus), "20000"], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "sanitized run ok" in r.stdout


def test_threaded_decoder_is_race_free(tmp_path):
    """ThreadSanitizer build of the same driver: the host decoder's thread pool over 40k-fragment
    batches (clean and mutated, both codecs, lenient and strict) reports no data race."""
    if not shutil.which("g++"):
        pytest.skip("no host C++ compiler")
    r = subprocess.run(["make", "-s", "-C", str(ROOT / "tools" / "sanitize"), "tsan"], capture_output=True, text=True)
    if r.returncode != 0 and "tsan" in (r.stderr or "").lower():
        pytest.skip("no ThreadSanitizer runtime: " + r.stderr[-300:])
    assert r.returncode == 0, r.stderr[-2000:]
    spans = gen_traces(72, 40, max_depth=4, anomalies=0.2)
    corpus = tmp_path / "corpus.bin"
    with open(corpus, "wb") as f:
        for s in spans:
            raw = T.span(s)
            for blob in (raw, T.snappy(raw)):
                f.write(struct.pack("<I", len(blob)) + blob)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    r = subprocess.run([str(BIN.parent / "fuzz_host_tsan"), str(corpus), "200"], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "sanitized run ok" in r.stdout
