set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/s1_tests.log 2>&1
rc=$?; tail -3 $OUT/s1_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/mb_launch_breakdown.py > $OUT/s1_mb_launches.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > $OUT/s1_bench.json 2> $OUT/s1_bench.err || exit $?
cat $OUT/s1_bench.json
