set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=gpurun_out/r6v; mkdir -p $O/jit
QSIM_JIT_DUMP=$R/$O/jit timeout -k 10 300 python -u bench.py --workload dm --steps 3 --warmup 1 > $O/dm.json 2> $O/dm.err || { tail -5 $O/dm.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/dm.json')); print('dm', d['value'], d['ms_per_step'])"
cd /tmp && timeout -s KILL 60 rocprofv3 --list-avail > $R/$O/avail.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_INSTS_VALU\b\|SQ_ACTIVE_INST_VALU\|SQ_WAIT_INST_ANY\|SQ_INST_CYCLES_VMEM\|SQ_WAVE_CYCLES\|SQ_BUSY_CYCLES\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_ANY\|SQ_ACTIVE_INST_ANY\|SQ_INSTS_SALU\|SQ_INSTS_LDS\|SQ_VALU_MFMA_BUSY_CYCLES\|SQ_INST_LEVEL_LDS" $R/$O/avail.txt | sort -u > $R/$O/names.txt || true
cat $R/$O/names.txt | tr '\n' ' '; echo
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $R/$O/pmc1 -o run --output-format csv -- python3 $R/bench.py --workload dm --steps 2 --warmup 1 > $R/$O/pmc1.log 2>&1 || { tail -5 $R/$O/pmc1.log; }
ls -R $R/$O/pmc1 | head -5
