#!/bin/bash
# FrameRing parity test, then the default bench at several frames-in-flight depths.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python3 -m pytest tests -m gpu -x -q -k "ring or device_path" > gpurun_out/ring_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/ring_pytest.log; [ $rc -eq 0 ] || exit $rc
for d in "$@"; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --frames-in-flight $d > gpurun_out/ring_b$d.json 2> gpurun_out/ring_b$d.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/ring_b$d.json'));print($d, d['value'], d['ms_per_step'], d['config']['frame_latency_ms'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])"
done
