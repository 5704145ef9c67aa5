"""ThreadSanitizer run of the library's concurrency code (SURVEY.md §5 "race detection: TSan on the
CPU build").

tests/tsan builds csrc/tfhe_api.cpp (key registry, per-thread lanes, the two-lane Tier-1
coalescing queue), csrc/multi.cpp (tfhe_gpu_init registry, per-device workers) and
csrc/circuit.cpp (per-context device state) UNCHANGED with -fsanitize=thread against a CPU
stand-in for the device engine (tests/tsan/stub_engine.cpp: the engine's locking discipline, a
deterministic stand-in for the gate arithmetic) and for the HIP host API (tests/tsan/stub/).
The driver hammers them: 64 threads of Tier-1 gate chains with results aliasing inputs and mixed
gate kinds (the reference's OpenMP callers, cpuParallel/Cipher.cpp:83-120, cloud.cpp:389-395);
tfhe_gpu_boots_batch from 8 threads on either device while tfhe_gpu_init re-registers the key and
other keys are imported, registered, used and deleted; one circuit run concurrently on contexts
that come and go.  Every result is compared word for word (current_variance bit for bit) with
the same work done sequentially, and DeviceScope's save / restore logic is unit-tested with the
stub's per-thread current device.  Pass = exit 0 and no ThreadSanitizer report."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
TSAN = os.path.join(HERE, "tsan")


def _tsan_available():
    return shutil.which("g++") is not None and shutil.which("make") is not None


@pytest.mark.skipif(not _tsan_available(), reason="needs g++ and make")
def test_concurrency_code_is_tsan_clean():
    subprocess.run(["make", "-s", "-j4", "-C", TSAN], check=True, timeout=600)
    exe = os.path.join(TSAN, "_bin", "tsan_driver")
    cmd = [exe, "64", "8"]
    # TSan maps its shadow memory at fixed addresses; without ASLR it never collides with a mapping
    if shutil.which("setarch"):
        cmd = ["setarch", os.uname().machine, "-R"] + cmd
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=0 exitcode=66 report_signal_unsafe=0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env)
    out = r.stdout + r.stderr
    assert "WARNING: ThreadSanitizer" not in out, out[-6000:]
    assert r.returncode == 0, out[-4000:]
    assert "tsan_driver: ok" in r.stdout
    for phase in ("tier1: 64 threads x 8 gates", "multi:", "circuits:"):
        assert phase in r.stdout, r.stdout
