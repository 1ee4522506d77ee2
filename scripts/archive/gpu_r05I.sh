# first-stream vs later-stream loop-top cycles of k_ingest_small at 1M / 125k streams (profiling build).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05I}
for S in 1000000 125000; do
  timeout -k 10 300 python tools/prof_sections.py --workload cfg3 --streams $S > gpurun_out/${TAG}_S$S.txt 2>&1 || { tail -5 gpurun_out/${TAG}_S$S.txt; exit 1; }
done
python3 - <<'PY'
import re
for S in (1000000, 125000):
    t = open('gpurun_out/r05I_S%d.txt' % S).read()
    vals = {int(m.group(1)): float(m.group(2)) for m in re.finditer(r'^\s+(\d+) .*?%\s+([0-9.e+]+)$', t, re.M)}
    print(S, ' '.join('%d:%.1fk' % (k, v / S / 1e3) for k, v in sorted(vals.items())), 'total %.1fk' % (sum(vals.values()) / S / 1e3),
          ' first-stream loop tops per wave: %.1fk' % (vals.get(11, 0) / 6144 / 1e3))
PY
