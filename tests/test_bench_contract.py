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


def test_gpus_flag_launches_one_rank_per_gpu(monkeypatch):
    """`bench.py --gpus N` outside a launcher re-runs itself under torch.distributed.run with N ranks (a
    child process, before any GPU call); inside a launch WORLD_SIZE must equal N."""
    import subprocess as sp

    import pytest
    sys.path.insert(0, ROOT)
    import bench
    seen = {}

    class Done:
        returncode = 7

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd
        return Done()

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sp, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-4:] == ["--gpus", "4", "--steps", "3"]
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.main()
