"""Run bench.py (argv passed through) and, from a Python atexit handler -- before the C-level
exit runs the shared libraries' destructors -- write this process's /proc/self/maps to
$TDS_MAPS_OUT, so an exit-time fault's PC can be placed in a library (gpu_sessions/r3_s15.sh)."""
import atexit
import os
import runpy
import sys

out = os.environ.get("TDS_MAPS_OUT", "maps.txt")


def _dump():
    with open("/proc/self/maps") as f, open(out, "w") as g:
        g.write(f.read())


atexit.register(_dump)
here = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, here)
sys.argv = [os.path.join(here, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
