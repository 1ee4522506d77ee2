# section cycles per stream without the fused stats role (GK_FUSED_STATS=0) at 1M / 125k streams.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05H}
for S in 1000000 125000; do
  GK_FUSED_STATS=0 timeout -k 10 300 python tools/prof_sections.py --workload cfg3 --streams $S > gpurun_out/${TAG}_S$S.txt 2>&1 || { tail -5 gpurun_out/${TAG}_S$S.txt; exit 1; }
  GK_FS_LAG=64 timeout -k 10 300 python tools/prof_sections.py --workload cfg3 --streams $S > gpurun_out/${TAG}_lag64_S$S.txt 2>&1 || { tail -5 gpurun_out/${TAG}_lag64_S$S.txt; exit 1; }
done
python3 - <<'PY'
import re
for tag in ("r05H_S", "r05H_lag64_S"):
    for S in (1000000, 125000):
        t = open('gpurun_out/%s%d.txt' % (tag, S)).read()
        vals = {int(m.group(1)): float(m.group(2)) for m in re.finditer(r'^\s+(\d+) .*?%\s+([0-9.e+]+)$', t, re.M)}
        print(tag, S, ' '.join('%d:%.1fk' % (k, v / S / 1e3) for k, v in sorted(vals.items())), 'total %.1fk' % (sum(vals.values()) / S / 1e3))
PY
