#!/bin/bash
# PMC passes over one bench leg (tools/leg_probe.py), per-kernel means for the kernels whose name holds <match>:
#   bash tools/pmc_leg.sh <out-dir> <leg> <match>
# Each pass is its own rocprofv3 process with counters only (no tracing domains); raw files stay in /tmp on the box.
set -o pipefail
out=$1; leg=$2; match=$3
mkdir -p "$out"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
raw=/tmp/mi_pmc_leg; rm -rf $raw; mkdir -p $raw
# PMC_SETS (optional): other counter sets, ';'-separated (each within one pass's per-block limits)
sets=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE"
      "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE"
      "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE")
[ -n "$PMC_SETS" ] && IFS=';' read -r -a sets <<< "$PMC_SETS"
i=0
for set in "${sets[@]}"; do
  i=$((i+1))
  echo "=== pass $i $(date +%T)"
  timeout -k 10 180 rocprofv3 --pmc $set --output-format csv -d $raw/p$i -o run -- python3 tools/leg_probe.py "$leg" 1 \
    > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$out/p$i.log"; exit 1; }
done
python3 - "$raw" "$match" > "$out/summary.txt" <<'PY'
import csv, glob, sys, collections
raw, match = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(raw + "/p*/run_counter_collection.csv"):
    for row in csv.DictReader(open(f)):
        if match in row["Kernel_Name"]:
            acc[row["Kernel_Name"][:70]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    print(k, " launches", max(len(v) for v in cs.values()))
    for c, v in sorted(m.items()):
        print(f"   {c:26s} {v:18.1f}")
    w = m.get("SQ_WAVES", 0)
    if w:
        print(f"   valu_per_wave              {m.get('SQ_INSTS_VALU', 0) / w:18.1f}")
        print(f"   lds_insts_per_wave         {m.get('SQ_INSTS_LDS', 0) / w:18.1f}")
    if m.get("SQ_BUSY_CYCLES"):
        print(f"   mfma_busy/busy             {m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / m['SQ_BUSY_CYCLES']:18.3f}")
    if m.get("TCC_HIT_sum") is not None and m.get("TCC_MISS_sum") is not None:
        t = m["TCC_HIT_sum"] + m["TCC_MISS_sum"]
        print(f"   l2_hit_rate                {m['TCC_HIT_sum'] / t if t else 0:18.3f}")
    if "FETCH_SIZE" in m:
        print(f"   hbm_fetch_bytes_corrected  {m['FETCH_SIZE'] * 2048:18.1f}")
PY
cat "$out/summary.txt"
