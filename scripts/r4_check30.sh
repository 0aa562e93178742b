cd "$GRAFT_REPO_ROOT"
bash scripts/r4_check20.sh || exit 1
bash scripts/r4_check29.sh || exit 1
