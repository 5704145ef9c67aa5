"""Tier-1 TFHE C API from many threads and in place: the reference's callers
enter the gates from OpenMP threads and pass results that alias inputs.  The driver
(tests/callers/tier1_threads.cpp) is built by __graft_entry__.build() through
tests/callers/Makefile against include/ + libtfhe_amd alone."""
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CALLERS = os.path.join(REPO, "tests", "callers")
EXE = os.path.join(CALLERS, "_bin", "tier1_threads")
LIB = os.path.join(REPO, "cpu-gpu-tfhe_amd", "lib", "libtfhe_amd.so")


@pytest.mark.skipif(not os.path.exists(LIB), reason="libtfhe_amd.so not built")
def test_tier1_driver_builds():
    """The driver compiles and links against the public headers and the library alone."""
    subprocess.check_call(["make", "-s", "-C", CALLERS])
    assert os.access(EXE, os.X_OK)


@pytest.mark.gpu
def test_tier1_threads_and_aliasing_gpu():
    """Every gate + MUX: sequential vs 8 OpenMP threads vs result aliasing an input give the
    same samples word for word, and every output decrypts to its truth table; 16 short-lived
    threads running one gate each leave the key's lane count unchanged."""
    assert os.access(EXE, os.X_OK), "tests/callers/_bin/tier1_threads missing: run __graft_entry__.build()"
    r = subprocess.run([EXE, "24"], capture_output=True, text=True, timeout=300)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, (r.returncode, r.stderr[-2000:])
    out = json.loads(lines[-1])
    assert r.returncode == 0, (out, r.stderr[-2000:])
    assert out["par_mismatch"] == 0 and out["alias_mismatch"] == 0 and out["truth_errors"] == 0, out
    # threads that exit give their lanes back (no stream / scratch / pinned-memory leak per thread)
    assert out["short_thread_errors"] == 0 and out["lanes_after_short_threads"] == out["lanes_before"], out
