#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT}"
for arm in pad nopad; do
  if [ $arm = nopad ]; then export AST_HIP_LIB=$R/build_var/libast_hip_nopad.so; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES --output-format csv -d "$R/gpurun_out/r04u_$arm" -o pmc -- python3 "$R/bench.py" --mode fwd --steps 2 --warmup 1 --cpu-seconds 0 > "$R/gpurun_out/r04u_$arm.log" 2>&1 || { echo "$arm failed"; exit 1; }
  echo "$arm ok"
done
