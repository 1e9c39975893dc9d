#!/bin/bash
# PMC passes over one large-N PBS shape leg (default 3_3): bash tools/pmc_shape.sh <out-dir> [shape]
# (A two-lane batch, >= 64 ciphertexts, crashes rocprofv3 --pmc on the host; pass a one-lane ad-hoc shape such as
# 8192,1,1077,15,2,48.)  Each pass its own rocprofv3 process (no tracing domains); per-kernel means (VALU per wave, issue-busy share, HBM
# bytes: FETCH_SIZE KiB x 2 on gfx950, WRITE_SIZE KiB) come back in <out-dir>/summary.txt, durations from a
# separate kernel trace.
set -o pipefail
out=${1:-gpurun_out/pmc_shape}; shape=${2:-message_3_carry_3}; mkdir -p "$out"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
raw=/tmp/mi_pmc_shape; rm -rf $raw; mkdir -p $raw
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $raw/trace -o run -- python3 tools/shape_probe.py $shape > "$out/trace.log" 2>&1 || { echo "trace failed"; exit 1; }
cp $raw/trace/run_kernel_stats.csv "$out/kernel_stats.csv"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  echo "=== pass $i $(date +%T)"
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d $raw/p$i -o run -- python3 tools/shape_probe.py $shape > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 - "$raw" > "$out/summary.txt" <<'PY'
import csv, glob, sys, collections
raw = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(raw + "/p*/run_counter_collection.csv"):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0][:80] + " grid=" + row["Grid_Size"]
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
rows = []
for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    n = max(len(v) for v in cs.values())
    rows.append((m.get("SQ_INSTS_VALU", 0) * n, k, m, n))
for _, k, m, n in sorted(rows, reverse=True)[:12]:
    w = m.get("SQ_WAVES", 0) or 1
    hbm = m.get("FETCH_SIZE", 0) * 2048 + m.get("WRITE_SIZE", 0) * 1024
    busy = m.get("SQ_ACTIVE_INST_VALU", 0) / max(1.0, m.get("SQ_WAVE_CYCLES", 1))
    print(f"{k}\n   dispatches {n}, waves {w:.0f}, VALU/wave {m.get('SQ_INSTS_VALU', 0) / w:.0f}, "
          f"active-VALU share of wave cycles {busy:.3f}, wait-inst share {m.get('SQ_WAIT_INST_ANY', 0) / max(1.0, m.get('SQ_WAVE_CYCLES', 1)):.3f}, "
          f"wait-any share {m.get('SQ_WAIT_ANY', 0) / max(1.0, m.get('SQ_WAVE_CYCLES', 1)):.3f}, HBM MB/dispatch {hbm / 1e6:.1f}")
PY
cat "$out/summary.txt"
