"""Config-5 inference step time at a given ops.INFER_TILE (the largest S tile, in triplets):
python scripts/c5_tile_probe.py TILE [bench args...] runs bench.py --workload aid_infer with it."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "x2-gnn_amd"))
from x2gnn import ops  # noqa: E402

ops.INFER_TILE = int(sys.argv[1])
sys.argv = [os.path.join(ROOT, "bench.py"), "--workload", "aid_infer", "--no-cpu-baseline"] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
