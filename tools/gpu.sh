#!/bin/bash
# One parameterised GPU-box pass (replaces the per-run gpu_r*.sh scripts of rounds 1-3).
#
#   tools/gpu.sh RUN STEP [STEP ...]
#
# writes everything under gpurun_out/RUN/ and runs the steps in order; each GPU step has a time
# limit of its own and the first failing step ends the pass (its log tail is printed).  STEP:
#   tests[:K]            pytest -m gpu, one process (K: a pytest -k expression; '+' for spaces)
#   smoke                __graft_entry__.smoke()
#   bench:NAME[:ARGS]    python bench.py ARGS  -> RUN/bench_NAME.log   (ARGS: ',' for spaces)
#   prof:NAME[:ARGS]     rocprofv3 --kernel-trace --stats of bench.py ARGS -> RUN/prof_NAME/
#   py:NAME:SCRIPT[:ARGS]  python SCRIPT ARGS -> RUN/NAME.log (probes under tools/)
#   pmc                  tools/pmc_passes.sh (PMC counter passes, one counter group per run)
# e.g. tools/gpu.sh r07a tests:drain smoke bench:c1 prof:c1:--steps,5,--no-cpu
set -o pipefail
export TMPDIR=/tmp
RUN=${1:?run name}
shift
OUT=gpurun_out/$RUN
mkdir -p "$OUT"

fail() {
  echo "FAILED: $1 (rc $2)"
  tail -c 4000 "$3"
  exit "$2"
}

for step in "$@"; do
  IFS=: read -r kind name rest <<< "$step"
  case "$kind" in
    tests)
      log=$OUT/pytest_gpu${name:+_$name}.log
      k=()
      [ -n "$name" ] && k=(-k "${name//+/ }")
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
        > "$log" 2>&1 || fail "$step" $? "$log"
      tail -n 1 "$log"
      ;;
    smoke)
      log=$OUT/smoke.log
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 || fail smoke $? "$log"
      tail -n 1 "$log"
      ;;
    bench)
      log=$OUT/bench_$name.log
      timeout -k 10 900 python -u bench.py ${rest//,/ } > "$log" 2>&1 || fail "$step" $? "$log"
      python tools/bench_summary.py "$log"
      ;;
    prof)
      log=$OUT/prof_$name.log
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$name" -o run \
        -- python3 bench.py ${rest//,/ } > "$log" 2>&1 || fail "$step" $? "$log"
      find "$OUT/prof_$name" -name "*kernel_stats*.csv" | sort
      ;;
    py)
      script=${rest%%:*}
      args=${rest#"$script"}
      args=${args#:}
      log=$OUT/$name.log
      timeout -k 10 600 python -u "$script" ${args//,/ } > "$log" 2>&1 || fail "$step" $? "$log"
      tail -n 20 "$log"
      ;;
    pmc)
      bash tools/pmc_passes.sh || exit $?
      ;;
    *)
      echo "unknown step $step"
      exit 2
      ;;
  esac
done
echo "pass $RUN done"
