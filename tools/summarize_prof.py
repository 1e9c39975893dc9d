#!/usr/bin/env python3
"""Turn a tools/profile_session.sh output directory into the committed profile artefacts.

  python tools/summarize_prof.py gpurun_out/prof_<tag> profiles/<tag>

Writes <dst>/kernel_stats.csv (rocprofv3 --kernel-trace --stats summary, copied), <dst>/pmc_summary.json
(per-kernel mean PMC values for the NTT transform kernels of the bench run, HBM bytes corrected as
MI355X_MICROARCH.md prescribes: FETCH_SIZE is in KiB and reports half the bytes of a coalesced
streaming read on gfx950 -> x1024 x2; WRITE_SIZE in KiB -> x1024) and refreshes
profiles/pmc_traffic.json, which bench.py reads for roofline.traffic.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ALG_BYTES = 8192 * 2048 * 8 * 2  # one N=2048 batch-8192 pass: read + write in place


def counters(path):
    vals = defaultdict(lambda: defaultdict(list))
    grid = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            k, g = row["Kernel_Name"], int(row["Grid_Size"])
            if "ntt" in k and g < 8192 * 64:  # transforms: only the full-batch launches (not the host-path ones)
                continue
            vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
            grid[k] = max(grid.get(k, 0), g)
    return vals, grid


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    if os.path.exists(os.path.join(src, "trace", "run_kernel_stats.csv")):  # (PMC-only sessions have no trace)
        shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    merged = defaultdict(dict)
    grids = {}
    for sub in ("pmc_sq", "pmc_lds", "pmc_fetch", "pmc_write"):
        p = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        vals, grid = counters(p)
        grids.update(grid)
        for k, cs in vals.items():
            for c, v in cs.items():
                merged[k][c] = sum(v) / len(v)
    summary = {}
    for k, cs in merged.items():
        if not any(t in k for t in ("ntt_window_kernel", "ntt_gl", "ntt_tw", "pbs_kernel", "pbs_tw_kernel", "pbs_tw_sol_kernel", "ext_tw_kernel", "bsk_to_ntt", "ext_product",
                                    "ks_gemm_kernel", "ks_digits_kernel")):
            continue
        if "ntt" in k and grids.get(k, 0) < 8192 * 64:  # only the full-batch launches
            continue
        d = dict(cs)
        if "FETCH_SIZE" in d:
            d["hbm_read_bytes_corrected"] = d["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in d:
            d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = d["hbm_read_bytes_corrected"] + d["hbm_write_bytes"]
            if "ntt" in k:
                d["algorithmic_bytes_per_launch"] = ALG_BYTES
        if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d and d["SQ_WAVES"]:
            d["valu_per_wave"] = d["SQ_INSTS_VALU"] / d["SQ_WAVES"]
        if "SQ_WAVE_CYCLES" in d and d["SQ_WAVE_CYCLES"]:
            for c in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in d:
                    d[c.lower() + "_per_wave_cycle"] = d[c] / d["SQ_WAVE_CYCLES"]
        if "SQ_INSTS_VALU" in d and d.get("GRBM_GUI_ACTIVE"):
            # GRBM_GUI_ACTIVE sums the 8 XCDs' cycles; SQ_ACTIVE_INST_VALU counts instructions on gfx950 (it equals
            # SQ_INSTS_VALU), so VALU issue-busy is instructions x the measured issue cost per instruction
            # (tools/valu_probe.hip; the bodies' mix averages 4.20 cycles) over the SIMD cycles
            simd_cycles = d["GRBM_GUI_ACTIVE"] / 8 * 1024
            d["valu_instr_per_simd_cycle"] = d["SQ_INSTS_VALU"] / simd_cycles
            if "ntt_tw" in k:
                d["valu_issue_busy"] = d["valu_instr_per_simd_cycle"] * 4.20
        summary[k] = d
    with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    ntt = {k: v for k, v in summary.items() if "ntt" in k and "hbm_bytes_per_launch" in v}
    if ntt:
        worst = max(ntt.items(), key=lambda kv: kv[1]["hbm_bytes_per_launch"])
        traffic = {"source": os.path.join(dst, "pmc_summary.json"), "kernel": worst[0],
                   "bytes_per_launch": worst[1]["hbm_bytes_per_launch"],
                   "per_kernel": {k: v["hbm_bytes_per_launch"] for k, v in ntt.items()}}
        root = os.path.dirname(os.path.abspath(dst.rstrip("/")))
        with open(os.path.join(root, "pmc_traffic.json"), "w") as f:
            json.dump(traffic, f, indent=1)
    for k, v in summary.items():
        print(k[:90], {c: round(x, 1) for c, x in v.items() if c in ("valu_per_wave", "hbm_bytes_per_launch", "SQ_LDS_BANK_CONFLICT")})


if __name__ == "__main__":
    main()
