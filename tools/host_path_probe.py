#!/usr/bin/env python3
"""bench.py's host-path leg alone (diagnostic): python tools/host_path_probe.py > host_path.json"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tfhe-rs-main_modified_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
import tfhe_ntt_amd as eng  # noqa: E402

print(json.dumps(bench.bench_host_path(eng, torch)), flush=True)
