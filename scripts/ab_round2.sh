#!/bin/bash
# Parity + A/B of the prepass lane-group configurations (RT_PREPASS_CFG) and the primary unit
# shapes (RT_UNIT_W builds librt_hip_U16 / _U32) against the default build.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab2
run_tests() { # $1 = label, rest = env settings
  local l=$1; shift
  env "$@" timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/ab2/t_$l.log 2>&1 || { echo "tests $l failed"; tail -5 gpurun_out/ab2/t_$l.log; exit 1; }
  echo "tests $l: $(tail -1 gpurun_out/ab2/t_$l.log)"
}
run_tests p1024_16 RT_PREPASS_CFG=1024,16
run_tests p512_8 RT_PREPASS_CFG=512,8
run_tests p256_4 RT_PREPASS_CFG=256,4
run_tests u16 RT_LIB_VARIANT=U16
run_tests u32 RT_LIB_VARIANT=U32
bash scripts/ab_bench.sh RT_PREPASS_CFG=0,0 RT_PREPASS_CFG=1024,16 RT_PREPASS_CFG=512,8 RT_PREPASS_CFG=1024,8 \
  RT_PREPASS_CFG=256,4 RT_LIB_VARIANT=U16 RT_LIB_VARIANT=U32 \
  RT_PREPASS_CFG=0,0 RT_PREPASS_CFG=1024,16 RT_PREPASS_CFG=512,8 RT_PREPASS_CFG=1024,8 RT_PREPASS_CFG=256,4 \
  RT_LIB_VARIANT=U16 RT_LIB_VARIANT=U32
