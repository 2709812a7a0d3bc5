set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06f_smoke.log 2>&1 || { tail -5 gpurun_out/r06f_smoke.log; exit 1; }
tail -2 gpurun_out/r06f_smoke.log
AST_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/r06f_bench2.json 2> gpurun_out/r06f_bench2.err || { tail -5 gpurun_out/r06f_bench2.err; exit 1; }
cat gpurun_out/r06f_bench2.json | cut -c1-300
AST_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --mode mobilenet --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/r06f_bench2mb.json 2> gpurun_out/r06f_bench2mb.err || { tail -5 gpurun_out/r06f_bench2mb.err; exit 1; }
cat gpurun_out/r06f_bench2mb.json | cut -c1-300
