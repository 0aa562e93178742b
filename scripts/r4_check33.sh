cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r4.log 2>&1 || { tail -20 gpurun_out/smoke_r4.log; exit 1; }
tail -2 gpurun_out/smoke_r4.log
bash scripts/r4_check20.sh || exit 1
