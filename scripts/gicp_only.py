"""Scan-registration bench alone (bench.py's scan_registration line)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

b = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
print(json.dumps(bench.scan_registration_bench(b)))
