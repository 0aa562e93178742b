cd "$GRAFT_REPO_ROOT"
bash scripts/r4_check18.sh || exit 1
bash scripts/r4_check17.sh || exit 1
bash scripts/r4_check13.sh || exit 1
