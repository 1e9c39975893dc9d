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


def _stub_leg(i, nested=False):
    leg = {"metric": "x" * 200, "value": 1.0e6 + i, "unit": "PBS/s", "steps": 1000, "ms_per_step": 1.2345678,
           "kernel_ms": 1.2, "ntt_equivalents_per_s": 4.0e9, "config": {"workload": "w" * 400},
           "roofline": {"bound": "valu", "frac": 0.912345678, "note": "n" * 400, "hbm": {"achieved": 1.0}},
           "cpu_baseline": {"value": 123.456789, "unit": "PBS/s", "cores": 16, "kind": "port", "sample": "s" * 300}}
    if nested:
        return {f"shape_{j}": dict(leg) for j in range(6)}
    return leg


def test_compact_line_fits_driver_tail():
    """the last stdout line is the compact record (<= 12 KB) with the headline, its roofline and
    CPU baseline, and one row per leg; the bulky record goes to a file. Worst case: every leg present, nested shape
    legs, long notes everywhere."""
    sys.path.insert(0, ROOT)
    import bench
    out = {"metric": "m", "value": 7.0e7, "unit": "fwd+inv NTT pairs/s", "n_gpus": 8, "steps": 10000, "warmup": 200,
           "ms_per_step": 0.117, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
           "data": "d" * 100,
           "config": {"workload": "w" * 200, "n": 2048, "batch_per_gpu": 8192, "global_batch": 65536,
                      "parallelism": "p" * 80, "hip_runtime": ["h" * 300] * 4,
                      "build": {"so_source_hash": "a" * 64, "tree_source_hash": "a" * 64, "match": True,
                                "so_path": "q" * 300}},
           "kernels": {"timed_launch_ms": 0.058, "fwd_ms": 0.057, "inv_ms": 0.06, "note": "n" * 300},
           "valu_bound": {"fwd": {"frac": 0.83, "model_ms": 1}, "inv": {"frac": 0.82}},
           "roofline": {"bound": "hbm", "achieved": 4600.0, "peak": 8000.0, "unit": "GB/s", "frac": 0.575,
                        "traffic": 269079430.4, "traffic_source": "t" * 300, "algorithmic_bytes_per_launch": 268435456,
                        "kernel": "ntt_tw_body_kernel"},
           "cpu_baseline": {"value": 1.6e6, "unit": "fwd+inv NTT pairs/s", "cores": 16, "kind": "port",
                            "sample": "s" * 250},
           "host_path": {"blob": "b" * 20000}, "default_stream": {"blob": "b" * 5000}}
    for i, name in enumerate(bench.LEG_ORDER):
        out[name] = _stub_leg(i, nested=name.startswith("pbs_shapes") or name == "plans")
    # config 5 at world 8: the sharded legs nested under pbs / pbs_fft reach the summary
    for name in ("pbs", "pbs_fft"):
        out[name]["sharded"] = dict(_stub_leg(90), scaling="strong", value_with_scatter_gather=2.5e5,
                                    ms_per_step_with_scatter_gather=300.123456, key_broadcast_ms=12.3,
                                    config={"global_batch": 65536, "n_gpus": 8, "transfer": "t" * 100})
    out["steady_state"] = {"value": 6.9e7, "steps": 8600, "seconds": 1.0012, "timed_launch_ms": 0.058,
                           "roofline_frac": 0.567, "note": "n" * 200}
    out["cold_start"] = {"value": 6.1e7, "ms_per_step": 0.13, "timed_launch_ms": 0.065, "roofline_frac": 0.51,
                         "note": "n" * 200}
    line = bench.compact_line(out, bench.FULL_RECORD)
    text = json.dumps(line)
    assert len(text.encode()) <= bench.LINE_MAX_BYTES, len(text)
    assert "\n" not in text
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config", "roofline",
              "cpu_baseline", "legs_summary"):
        assert k in line, k
    assert line["roofline"]["frac"] == 0.575 and line["cpu_baseline"]["value"] == 1.6e6
    for name in ("pbs", "pbs_solinas", "ext_product"):
        row = line["legs_summary"][name]
        assert {"value", "ms_per_step", "steps", "frac", "alg_frac"} <= set(row), row
    assert "host_path" not in line and "hip_runtime" not in line["config"]
    for name in ("pbs.sharded", "pbs_fft.sharded"):
        row = line["legs_summary"][name]
        assert {"value", "value_with_scatter_gather", "ms_per_step", "ms_per_step_with_scatter_gather", "steps",
                "scaling"} <= set(row), row
    assert line["steady_state"]["roofline_frac"] == 0.567 and line["steady_state"]["seconds"] == 1.0012
    assert line["cold_start"]["value"] == 6.1e7
    assert line["roofline"]["traffic_source"]


def test_compact_line_of_last_rounds_full_record():
    """The real round-4 record (21 KB on one line, unparsed by the driver) compacts under the bound."""
    import pytest
    sys.path.insert(0, ROOT)
    import bench
    path = os.path.join(ROOT, "profiles", "r4", "session26", "bench_line.json")
    if not os.path.exists(path):
        pytest.skip("round-4 record not in this tree")
    out = json.load(open(path))
    text = json.dumps(bench.compact_line(out, bench.FULL_RECORD))
    assert len(text.encode()) <= 6 * 1024, len(text)
