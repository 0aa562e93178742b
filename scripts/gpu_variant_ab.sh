#!/bin/bash
# One GPU call for an experiment build: the -m gpu tests against the variant library
# (_build/librt_hip_<variant>.so), then a same-box A/B of the default bench against the product
# library, alternating.  usage: gpu_variant_ab.sh <variant> [pytest -k expression]
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=$1
K=${2:-}
RT_LIB_VARIANT=$V timeout -k 10 600 python3 -u scripts/with_variant.py -m pytest tests -m gpu -x -q \
  --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/${V}_tests.log 2>&1 \
  || { tail -30 gpurun_out/${V}_tests.log; exit 1; }
tail -1 gpurun_out/${V}_tests.log
bash scripts/ab_bench.sh RT_LIB_VARIANT= RT_LIB_VARIANT=$V RT_LIB_VARIANT= RT_LIB_VARIANT=$V
