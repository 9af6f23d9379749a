"""Run bench.py against a variant library (tools/build_variants.sh); diagnostic only."""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import rl4co_slap_amd._native as nat  # noqa: E402

nat.LIB_PATH = sys.argv[1]
sys.argv = ["bench.py"] + sys.argv[2:]
runpy.run_path("bench.py", run_name="__main__")
