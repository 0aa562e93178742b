#!/bin/bash
# HBM bytes per tracescreen launch of the default bench (one batch in flight): FETCH_SIZE and
# WRITE_SIZE passes only, then the same summary profile_round.sh gives (traffic.json).
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/traffic; rm -rf $O; mkdir -p $O
# STEPS=10: one 10-frame launch, the batch of the driver's `bench.py --steps 20` run
STEPS=${STEPS:-12}
pmc() { local n=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o run -- python3 bench.py --steps $STEPS --warmup 1 --no-cpu-baseline --traffic off --no-companions --frames-in-flight 1 > $O/$n.log 2>&1; local rc=$?; echo "pmc $n rc=$rc"; return $rc; }
pmc fetch FETCH_SIZE && pmc write WRITE_SIZE
