"""Progress lines of long GPU tests: to stderr and, when the repo has a gpurun_out/ directory (the
GPU box's copy does), appended to gpurun_out/progress.log -- pytest captures stderr until a test
ends, and a GPU command whose outputs stay silent for minutes is taken for hung."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_T0 = time.time()


def say(what, t0=None):
    line = f"[{time.strftime('%H:%M:%S')} +{time.time() - (t0 or _T0):7.1f}s pid {os.getpid()}] {what}"
    print(line, file=sys.stderr, flush=True)
    d = os.path.join(REPO, "gpurun_out")
    if os.path.isdir(d):
        with open(os.path.join(d, "progress.log"), "a") as f:
            f.write(line + "\n")
