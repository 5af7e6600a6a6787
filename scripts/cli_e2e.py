"""bench.py's cli_end_to_end extra on its own (one JSON line): the whole CLI on 2M reads from an
hg19-shaped genome, BAM on a stdin pipe and SAM by path, with the process phases from run.log."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    print(json.dumps(bench.cli_end_to_end(n)), flush=True)
