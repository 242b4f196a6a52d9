#!/bin/bash
# Config 2 sustained: 20 000 back-to-back steps while rocm-smi samples clocks / power every ~0.5 s (read-only).
set -o pipefail
out=gpurun_out/clk
mkdir -p $out
( for i in $(seq 1 150); do date +%s.%N; timeout -k 2 5 rocm-smi --showclocks --showpower --showtemp 2>&1 | grep -E "sclk|mclk|fclk|Power|Temperature \(Sensor (junction|memory)" ; sleep 0.3; done ) > $out/smi.log 2>&1 &
smi=$!
date +%s.%N > $out/bench_start
timeout -k 10 240 python3 bench.py --steps 20000 --warmup 50 --no-config4 --no-cpu-baseline --no-verify > $out/bench.json 2> $out/bench.err
rc=$?
date +%s.%N > $out/bench_end
kill $smi 2>/dev/null
wait $smi 2>/dev/null
python3 scripts/show_bench.py $out/bench.json || true
exit $rc
