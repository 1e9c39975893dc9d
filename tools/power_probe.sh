#!/bin/bash
# sample power/clock while the transform probe runs
mkdir -p gpurun_out
( for i in $(seq 1 12); do rocm-smi --showpower --showclocks --showtemp 2>/dev/null | grep -E "Power|sclk|mclk|fclk|Temperature|socclk" ; echo ---; sleep 0.5; done ) > gpurun_out/power_samples.txt 2>&1 &
SP=$!
timeout -k 10 200 ./tools/variant_probe 8192 > gpurun_out/variants_p.txt 2>&1
wait $SP
rocm-smi --showpower --showmaxpower 2>/dev/null | grep -iE "power" >> gpurun_out/power_samples.txt
