cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r03v
bash scripts/gpu_ab.sh $TAG "GK_FS_LAG=256" "GK_FS_LAG=64" "GK_FS_LAG=128" "GK_FS_LAG=32" "GK_FS_LAG=256" || exit 1
bash scripts/pmc_fetch_ab.sh $TAG "GK_FS_LAG=256" "GK_FS_LAG=128" "GK_FS_LAG=64" "GK_FS_LAG=32" || exit 1
