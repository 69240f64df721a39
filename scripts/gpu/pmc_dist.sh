# PMC HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the sharded engine's local pass
# kernels at the shard size of a W-rank run of W-HC 30q: W virtual shards on one GPU run the same
# planner, per-rank lowering and kernels as the RCCL ranks (exchanges as device copies), so the
# per-launch bytes of its pass kernels are those of one rank's.  -> profiles/pmc_dist_hc_30q_<W>.json
#     gpurun --timeout 1200 -- bash scripts/gpu/pmc_dist.sh <tag> [worlds...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/${1:-pmc_dist}
shift
WORLDS=${*:-8 4 2}
mkdir -p $O
for w in $WORLDS; do
  for i in 1 2; do
    C=FETCH_SIZE; [ $i = 2 ] && C=WRITE_SIZE
    cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $C -d $O/pmc_dist_$w/p$i -o run --output-format csv -- python3 $R/scripts/dist_virtual_bench.py 30 $w 2 > $O/pmc_dist_${w}_p$i.log 2>&1 || { cd $R; tail -5 $O/pmc_dist_${w}_p$i.log; exit 1; }
    cd $R
  done
  python3 scripts/pmc_summary.py $O/pmc_dist_$w $O/pmc_dist_hc_30q_$w.json > $O/pmc_dist_hc_30q_$w.txt || exit 1
  head -12 $O/pmc_dist_hc_30q_$w.txt
done
