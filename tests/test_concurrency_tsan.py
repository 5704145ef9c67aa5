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
stub's per-thread current device.  Pass = exit 0 and no ThreadSanitizer report.

Round 5: csrc/engine.cpp itself is built the same way (tests/tsan/_bin/tsan_engine:
the whole host library + CPU stand-in kernels, tests/tsan/stub_kernels.cpp) against a stub HIP
runtime whose streams are asynchronous worker threads, so a host read that is not ordered after
the stream work producing it is a race TSan sees.  tsan_engine_driver.cpp hammers the host copy
pool from three contexts (two devices, one a key replica built meanwhile), several threads on one
context at once, over the staged, sliced, record (LweSample rows + device current_variance) and
caller-owned pinned paths, plus the pinned registry under alloc / free churn; every result is
compared word for word with a sequential run.  A mutation check proves the harness can fail: the
same build with the pinned path's final stream synchronization deleted must draw a TSan report."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
TSAN = os.path.join(HERE, "tsan")


def _run(exe, *args):
    cmd = [exe, *map(str, args)]
    # TSan maps its shadow memory at fixed addresses; without ASLR it never collides with a mapping
    if shutil.which("setarch"):
        cmd = ["setarch", os.uname().machine, "-R"] + cmd
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=0 exitcode=66 report_signal_unsafe=0")
    return subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env)


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


@pytest.mark.skipif(not _tsan_available(), reason="needs g++ and make")
def test_engine_host_side_is_tsan_clean():
    subprocess.run(["make", "-s", "-j4", "-C", TSAN, "_bin/tsan_engine"], check=True, timeout=600)
    r = _run(os.path.join(TSAN, "_bin", "tsan_engine"), 8, 2)
    out = r.stdout + r.stderr
    assert "WARNING: ThreadSanitizer" not in out, out[-6000:]
    assert r.returncode == 0, out[-4000:]
    assert "tsan_engine_driver: ok" in r.stdout
    for phase in ("sequential: 10 workloads", "engine host paths: 8 threads", "all equal", "pinned registry:"):
        assert phase in r.stdout, r.stdout


@pytest.mark.skipif(not _tsan_available(), reason="needs g++ and make")
def test_engine_tsan_harness_catches_a_missing_synchronization():
    """Mutation check: without the pinned host path's hipStreamSynchronize the host reads results the
    (asynchronous) stub stream is still writing — the harness must report it."""
    src = open(os.path.join(HERE, "..", "cpu-gpu-tfhe_amd", "csrc", "engine.cpp")).read()
    cut = "    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);\n    tr.lap(tr.wait);\n"
    assert src.count(cut) == 1, "the pinned path's final synchronization moved: update the mutation"
    os.makedirs(os.path.join(TSAN, "_bin"), exist_ok=True)
    mut = "// engine.cpp with the pinned path's final stream synchronization removed (mutation check)\n" + \
        src.replace(cut, "    tr.lap(tr.wait);\n")
    path = os.path.join(TSAN, "_bin", "engine_mut.cpp")
    if not os.path.exists(path) or open(path).read() != mut:
        open(path, "w").write(mut)
    subprocess.run(["make", "-s", "-j4", "-C", TSAN, "_bin/tsan_engine_mut"], check=True, timeout=600)
    r = _run(os.path.join(TSAN, "_bin", "tsan_engine_mut"), 4, 1)
    assert "WARNING: ThreadSanitizer" in r.stdout + r.stderr and r.returncode != 0
