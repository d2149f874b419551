"""Dev rehearsal: run bench.py's N-rank pipeline with every rank on GPU 0
(the box has one GPU; RCCL refuses two ranks on one device, so use
--dist-backend gloo). Sets LOCAL_RANK=0 for bench.py's device choice."""
import os
import runpy
import sys

os.environ["LOCAL_RANK"] = "0"
sys.argv = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
