set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TUNE_CIN3=1 TUNE_CFGS=12,18,19,20,21,22,23,42,43 TUNE_COPY=gpurun_out/r06c3_tuning.json
for m in "" TUNE_TRAIN TUNE_AE TUNE_AST; do
  echo "== fwd ${m:-bench}"
  env ${m:+$m=1} timeout -k 10 300 python3 -u scripts/tune_conv.py >> gpurun_out/r06c3_tune.log 2>&1 || { tail -5 gpurun_out/r06c3_tune.log; exit 1; }
done
for d in train ast ae; do
  echo "== dgrad $d"
  TUNE_DGRAD=$d timeout -k 10 300 python3 -u scripts/tune_conv.py >> gpurun_out/r06c3_tune.log 2>&1 || { tail -5 gpurun_out/r06c3_tune.log; exit 1; }
done
grep shape gpurun_out/r06c3_tune.log | cut -c1-200
