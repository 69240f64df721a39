# round 6: register-stage beam + stage-weighted DM candidates (DM 14q, W-HC 30q)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6c; mkdir -p $O
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload dm --steps 5 --warmup 1 > $O/dm_$tag.json 2> $O/dm_$tag.err || { tail -5 $O/dm_$tag.err; return 1; }
  python3 -c "
import json; d=json.load(open('$O/dm_$tag.json')); print('$tag dm', d['value'], d['ms_per_step'], d['passes'], d['roofline']['frac'])"
}
run b0w0t256 QSIM_STAGE_BEAM=0 QSIM_DM_STAGE_US=0 || exit 1
run b4w1k QSIM_STAGE_BEAM=4 QSIM_DM_STAGE_US=1000 || exit 1
run b4w1kt1024 QSIM_STAGE_BEAM=4 QSIM_DM_STAGE_US=1000 QSIM_DM_RELABEL_TRIES=1024 || exit 1
run b16w1kt1024 QSIM_STAGE_BEAM=16 QSIM_DM_STAGE_US=1000 QSIM_DM_RELABEL_TRIES=1024 || exit 1
run b4w0 QSIM_STAGE_BEAM=4 QSIM_DM_STAGE_US=0 || exit 1
for b in 4 0; do
  QSIM_STAGE_BEAM=$b timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-1q28 --no-batch16 --no-extras --cpu-budget 0 > $O/hc_b$b.json 2> $O/hc_b$b.err || { tail -5 $O/hc_b$b.err; exit 1; }
  python3 -c "
import json; h=json.load(open('$O/hc_b$b.json')); print('beam $b hc', h['value'], h['ms_per_step'], h['config']['passes'], h['roofline']['frac'])"
done
