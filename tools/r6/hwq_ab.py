"""Run bench.py with the hardware-queue floor taken out (GPU_MAX_HW_QUEUES as exported),
for a same-box A/B of the queue count on the batch lines.  Usage (repo root):
python tools/r6/hwq_ab.py <bench args...>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src = open(os.path.join(ROOT, "bench.py")).read()
floor = 'if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:\n    os.environ["GPU_MAX_HW_QUEUES"] = "8"\n'
assert floor in src
src = src.replace(floor, "")
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
g = {"__name__": "__main__", "__file__": sys.argv[0]}
exec(compile(src, sys.argv[0], "exec"), g)
