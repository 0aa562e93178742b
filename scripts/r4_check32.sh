cd "$GRAFT_REPO_ROOT"
bash scripts/r4_check31.sh || exit 1
bash scripts/r4_check13.sh || exit 1
