#!/bin/bash
# Parity tests of the default build (a -k selection), then the bench A/B of variant libraries
# (gpgpuraytrace_amd/_build/librt_hip_<name>.so; "" = default), each setting twice, interleaved.
# usage: TESTK="golden or baseline_config" ab_variants.sh p0 p2
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTK:-frame_bitexact_device_path or baseline_config}" \
  > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
set_list="RT_LIB_VARIANT="
for v in "$@"; do set_list="$set_list RT_LIB_VARIANT=$v"; done
bash scripts/ab_bench.sh $set_list $set_list
