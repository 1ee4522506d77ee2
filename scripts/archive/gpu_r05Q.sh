# wg flush cost presorted vs unsorted (one 10^7 stream alone; GK_WG_PRESORT=0: every batch ranked among its gaps' members)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for ps in 1 0; do
  GK_WG_PRESORT=$ps timeout -k 10 120 python tools/wg_alone.py 1 10000000 3 2>&1 | grep "per flush" | sed "s/^/presort=$ps /"
  GK_WG_PRESORT=$ps timeout -k 10 120 python tools/wg_alone.py 23 10000000 2 2>&1 | grep "per flush" | sed "s/^/presort=$ps /"
done
