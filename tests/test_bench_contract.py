"""bench.py's VALU issue model constants stay in sync with the generated bodies (no GPU)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_valu_cycles_match_generators():
    sys.path.insert(0, ROOT)
    import bench
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "valu_cost.py")], check=True,
                         capture_output=True, text=True).stdout
    model = json.loads(out)
    for k, v in bench.VALU_CYCLES.items():
        assert abs(model[k] - v) < 0.5, (k, model[k], v)
    assert not any(k.endswith("_unpriced") for k in model), model
