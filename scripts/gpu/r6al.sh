set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r6al; mkdir -p $O
for X in 1 0 3 5 7 -1; do
  cd /tmp && QSIM_JIT_XCD=$X timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/x$X -o run -- python3 $R/bench.py --steps 6 --warmup 2 --no-extras --no-1q28 --no-batch16 --cpu-budget 0 > $O/x$X.json 2> $O/x$X.err || { tail -5 $O/x$X.err; exit 1; }
  cd $R
  python3 - <<PY
import csv, json, glob
d=json.load(open('$O/x$X.json'))
f=glob.glob('$O/x$X/**/run_kernel_stats.csv', recursive=True)
rows=list(csv.DictReader(open(f[0]))) if f else []
print('xcd $X', d['value'], d['ms_per_step'], sorted([(r['Name'][:8], int(r['Calls']), round(float(r['AverageNs'])/1e6,3)) for r in rows if r['Name'].startswith('qk')]))
PY
done
