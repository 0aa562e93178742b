#!/bin/bash
# Round 6's final measurements in one gpurun call (gpurun_out/r6final/): every GPU test, smoke, the driver's bench
# command, the C1 / C2 / C5 configs and rocprofv3 --kernel-trace --stats over the driver's command.
#   gpurun -- bash scripts/measure_r06.sh
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_run.sh r6final testsall smoke "bench=--gpus 1 --steps 20 --warmup 5" "bench=--config c1" \
  "bench=--config c2" "bench=--config c5 --cpu-row-step 16" "prof=--gpus 1 --steps 20 --warmup 5"
