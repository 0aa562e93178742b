#!/bin/bash
# GPU round trip: parity tests, a short bench, and a kernel-trace profile.
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/check; mkdir -p $O
timeout -k 10 400 python3 -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1 && tail -1 $O/bench.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/kt.log 2>&1 && echo kt ok
