#!/bin/bash
# Quick PMC passes for the NTT kernels: bash tools/pmc_quick.sh <tag>
set -o pipefail
tag=${1:-q}
out=gpurun_out/pmc_$tag; mkdir -p $out
export PYTHONUNBUFFERED=1
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAIT_ANY" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $set --output-format csv -d $out/p$i -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pbs > $out/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/run_counter_collection.csv"):
    for row in csv.DictReader(open(f)):
        if "ntt" in row["Kernel_Name"] and int(row["Grid_Size"]) >= 8192 * 64:
            acc[row["Kernel_Name"][:60]][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v)/len(v):16.1f}")
PY
