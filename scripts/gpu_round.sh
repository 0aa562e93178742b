#!/bin/bash
# One GPU call for a candidate build: its parity tests, an A/B of the default bench against the
# default build, then the round profile of the default build and an instruction-cache PMC pass.
# usage: gpu_round.sh <variant>   (gpgpuraytrace_amd/_build/librt_hip_<variant>.so)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=$1
RT_LIB_VARIANT=$V timeout -k 10 400 python3 -u scripts/with_variant.py -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${V}_tests.log 2>&1 || { tail -5 gpurun_out/${V}_tests.log; exit 1; }
tail -1 gpurun_out/${V}_tests.log
bash scripts/ab_bench.sh RT_LIB_VARIANT= RT_LIB_VARIANT=$V RT_LIB_VARIANT= RT_LIB_VARIANT=$V || exit 1
bash scripts/profile_round.sh > gpurun_out/profile_round.log 2>&1 || { tail -5 gpurun_out/profile_round.log; exit 1; }
tail -3 gpurun_out/profile_round.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
  --output-format csv -d gpurun_out/icache -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --traffic off \
  --frames-in-flight 1 > gpurun_out/icache.log 2>&1
echo "icache pass rc=$?"
