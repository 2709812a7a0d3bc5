#!/bin/bash
# The one GPU-box session script (replaces the round-3 one-off gpu_r3*.sh files). Usage:
#   gpurun -- bash scripts/gpu.sh TAG TASK [TASK ...]
# Tasks run in order; the session stops at the first task that fails (a test failure inside
# `tests` is recorded and does not stop it; a timeout, abort or crash does). Outputs go to
# gpurun_out/TAG_*. Tasks:
#   tests            the -m gpu suite (no -x; per-test timeout)
#   tests:EXPR       the -m gpu tests matching -k EXPR
#   bench            bench.py default line (config 2, with its CPU baseline, as the driver runs it)
#   bench:MODE       bench.py --mode MODE (no CPU baseline): train, mobilenet, ast-train, ae-train
#   profiles         rocprofv3 kernel-trace stats + FETCH/WRITE_SIZE passes (scripts/measure_profiles.sh)
#   clock            effective clock and MFMA busy of the config-2 conv dispatches (scripts/pmc_clock.sh)
#   race             scripts/debug/race_probe4.py (16 repeats) and dp_repeat.py (8 runs) beside a
#                    background config-3 bench (the concurrent-load condition of DESIGN.md §4)
#   race:idle        the same probes with no background load
#   race:split       the same with the probes and the load on disjoint CU halves (HSA_CU_MASK)
#   py:SCRIPT[:ARGS] python3 SCRIPT ARGS (comma-separated), 300 s limit
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT=gpurun_out; mkdir -p $OUT
TAG="$1"; shift

run_tests() {
  local k="$1" log=$OUT/${TAG}_tests${2:-}.log
  timeout -k 10 900 python -u -m pytest tests -m gpu ${k:+-k "$k"} -q -p no:cacheprovider --timeout 300 \
      --timeout-method thread > $log 2>&1
  local rc=$?
  grep -E "^FAILED|^ERROR|passed|failed" $log | tail -12
  [ $rc -le 1 ]
}

run_race() {
  local LP=""
  if [ "$1" = "load" ]; then
    env ${LOAD_CU_MASK:+HSA_CU_MASK=$LOAD_CU_MASK} timeout -k 10 420 python3 bench.py --mode train --steps ${LOAD_STEPS:-1500} \
        --warmup 2 --cpu-seconds 0 > $OUT/${TAG}_race_load$2.json 2>&1 &
    LP=$!
    sleep 20
  fi
  env ${PROBE_CU_MASK:+HSA_CU_MASK=$PROBE_CU_MASK} timeout -k 10 150 python3 -u scripts/debug/race_probe4.py ${PROBE_N:-16} $OUT \
      > $OUT/${TAG}_race_probe4$2.txt 2>&1
  local rc=$?
  if [ $rc -eq 0 ] && [ "${DP_RUNS:-8}" -gt 0 ]; then
    env ${PROBE_CU_MASK:+HSA_CU_MASK=$PROBE_CU_MASK} timeout -k 10 240 python3 -u scripts/debug/dp_repeat.py ${DP_RUNS:-8} /tmp \
        > $OUT/${TAG}_dp_repeat$2.txt 2>&1
    rc=$?
  fi
  [ -n "$LP" ] && { kill $LP 2>/dev/null; wait $LP 2>/dev/null; }
  grep -v amdgpu.ids $OUT/${TAG}_race_probe4$2.txt | grep -E "FIRST|repeats differ" | head -20
  [ -f $OUT/${TAG}_dp_repeat$2.txt ] && grep -E "worst" $OUT/${TAG}_dp_repeat$2.txt
  return $rc
}

for task in "$@"; do
  echo "== $task"
  case "$task" in
    tests) run_tests "" || exit 1 ;;
    tests:*) run_tests "${task#tests:}" "_k" || exit 1 ;;
    bench)
      timeout -k 10 300 python bench.py > $OUT/${TAG}_bench_fwd.json 2> $OUT/${TAG}_bench_fwd.err || exit 1
      cut -c1-400 $OUT/${TAG}_bench_fwd.json ;;
    bench:*)
      m="${task#bench:}"
      timeout -k 10 300 python bench.py --mode $m --cpu-seconds 0 > $OUT/${TAG}_bench_$m.json 2> $OUT/${TAG}_bench_$m.err || exit 1
      cut -c1-400 $OUT/${TAG}_bench_$m.json ;;
    profiles) bash scripts/measure_profiles.sh ${TAG}m || exit 1 ;;
    clock) bash scripts/pmc_clock.sh ${TAG} fwd conv3x3 > $OUT/${TAG}_clock.txt 2>&1; rc=$?; cat $OUT/${TAG}_clock.txt; [ $rc -eq 0 ] || exit 1 ;;
    race) run_race load "" || exit 1 ;;
    race:idle) run_race idle _idle || exit 1 ;;
    race:split)  # the probes on CUs 0-127, the load on CUs 128-255 (HSA_CU_MASK): no CU shared
      LOAD_CU_MASK=0:128-255 PROBE_CU_MASK=0:0-127 run_race load _split || exit 1 ;;
    py:*)
      spec="${task#py:}"; script="${spec%%:*}"; args=""
      [ "$spec" != "$script" ] && args="${spec#*:}"
      timeout -k 10 300 python3 -u $script ${args//,/ } > $OUT/${TAG}_$(basename $script .py).txt 2>&1
      rc=$?; tail -30 $OUT/${TAG}_$(basename $script .py).txt; [ $rc -eq 0 ] || exit 1 ;;
    *) echo "unknown task $task"; exit 2 ;;
  esac
done
