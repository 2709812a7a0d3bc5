set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python scripts/bench_mb_blocks.py 32 dec10 > gpurun_out/pmc5_blk.log 2>&1 || exit $?
cat gpurun_out/pmc5_blk.log | grep -v amdgpu
PMC_KERNEL=expand_dw4 bash scripts/pmc_kernel.sh pmc5 scripts/bench_mb_blocks.py 8 dec10
PMC_KERNEL=expand_dw4 bash scripts/pmc_kernel.sh pmc3 scripts/bench_mb_blocks.py 8 enc1
