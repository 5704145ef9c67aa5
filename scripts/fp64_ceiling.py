"""fp64 FMA rate the GPU sustains (dev tool, GPU box): tfhe_amd_fp64_ceiling at 1, 2, 4, 8 waves
per SIMD, each for ~4 s, with amd-smi socket power / GFX clock sampled meanwhile."""
import re
import subprocess
import sys
import threading
import time

sys.path.insert(0, "cpu-gpu-tfhe_amd")
import tfhe_amd as T  # noqa: E402


def sample(stop, out):
    while not stop.is_set():
        try:
            txt = subprocess.run(["amd-smi", "metric", "-g", "0", "--clock", "--power"], capture_output=True,
                                 text=True, timeout=5).stdout
            w = re.findall(r"SOCKET_POWER:\s*([0-9.]+)", txt)
            if w:
                out.append(float(w[0]))
        except Exception:
            pass
        time.sleep(0.5)


for wps in (1, 2, 4, 8):
    stop, watts = threading.Event(), []
    th = threading.Thread(target=sample, args=(stop, watts))
    th.start()
    time.sleep(0.3)
    tf, mhz = T.fp64_ceiling(0, wps, 4.0)
    stop.set()
    th.join()
    busy = [w for w in watts if w > 400] or [0.0]
    print("waves/SIMD %d: %.1f TFLOP/s  %.0f MHz  %.0f W (%d samples)" % (wps, tf, mhz, sum(busy) / len(busy), len(busy)),
          flush=True)
