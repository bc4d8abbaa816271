#!/bin/bash
# Host-side scan probes on the GPU box's CPUs (no GPU use): the instrumented scan's per-phase
# cycles (varlib/hp_instr.so, built from csrc/hostpack.cpp with rdtsc stamps) at 1 and 16
# threads, and the scan switches A/B.  usage: tools/host_probe.sh RUN
set -o pipefail
OUT=gpurun_out/$1
mkdir -p "$OUT"
for t in 1 16; do
  EDV_SCAN_PROFILE=1 HOSTPACK_SO=varlib/hp_instr.so timeout -k 10 300 python tools/scan_cpu_bench.py 1000000 $t 3 \
    > "$OUT/scan_instr_t$t.log" 2>&1 || exit $?
done
timeout -k 10 400 python tools/scan_probe.py 1000000 1,8,16 5 EDV_SCAN_SHAPES=1/0 EDV_SCAN_PREFETCH=1/0 \
  > "$OUT/scan_probe.log" 2>&1 || exit $?
tail -n 12 "$OUT/scan_probe.log"
