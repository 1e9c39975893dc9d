#!/bin/bash
# Quick PMC passes for the headline NTT kernels: bash tools/pmc_quick.sh <out-dir>
# Each pass is its own rocprofv3 process (no tracing domains); the raw counter files stay in /tmp on the box, the
# per-kernel means come back in <out-dir>/summary.txt (LDS bank conflicts, VALU per wave, HBM bytes: FETCH_SIZE is
# KiB and half the coalesced-read bytes on gfx950 -> x1024 x2; WRITE_SIZE KiB -> x1024, MI355X_MICROARCH.md).
set -o pipefail
out=${1:-gpurun_out/pmc_q}; mkdir -p "$out"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
raw=/tmp/mi_pmc; rm -rf $raw; mkdir -p $raw
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAIT_ANY" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  echo "=== pass $i $(date +%T)"
  timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d $raw/p$i -o run -- python3 bench.py --steps 3 --warmup 1 \
    --no-cpu-baseline --no-pbs --no-shapes > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 - "$raw" > "$out/summary.txt" <<'PY'
import csv, glob, sys, collections
raw = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(raw + "/p*/run_counter_collection.csv"):
    for row in csv.DictReader(open(f)):
        if "ntt_tw_body_kernel" in row["Kernel_Name"] and int(row["Grid_Size"]) == 8192 * 64:
            acc[row["Kernel_Name"][:60]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k)
    for c, v in sorted(m.items()):
        print(f"   {c:24s} {v:16.1f}")
    w = m.get("SQ_WAVES", 0)
    if w:
        print(f"   valu_per_wave            {m.get('SQ_INSTS_VALU', 0) / w:16.1f}")
        print(f"   lds_insts_per_wave       {m.get('SQ_INSTS_LDS', 0) / w:16.1f}")
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        print(f"   hbm_bytes_corrected      {m['FETCH_SIZE'] * 2048 + m['WRITE_SIZE'] * 1024:16.1f}  (algorithmic 268435456)")
PY
cat "$out/summary.txt"
