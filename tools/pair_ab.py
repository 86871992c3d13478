"""bench.py with the persistent encoder-pair kernels forced on or off (A/B of
ops.PAIR_PERSISTENT; every other argument goes to bench.py):
python tools/pair_ab.py on|off [bench args]"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module("s-cgib_amd")
pkg.ops.PAIR_PERSISTENT = sys.argv[1] == "on"
sys.argv = ["bench.py"] + sys.argv[2:]
import bench  # noqa: E402

bench.main()
