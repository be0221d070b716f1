set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcw
cd /root/repo
for P in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_REQ_sum" "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  tag=$(echo $P | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/pmcw/$tag -o pmc -- python3 tools/opbench.py --iters 3 --wide 1 2 --only gemm_geglu_1280 gemm_geglu_320 > gpurun_out/pmcw/$tag.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for d in sorted(glob.glob('gpurun_out/pmcw/*/')):
    rows=[]
    for f in glob.glob(d+'**/*counter_collection.csv', recursive=True):
        rows+=list(csv.DictReader(open(f)))
    agg=collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        k=r['Kernel_Name'][:60]
        agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
    print('==', d)
    for k,v in agg.items():
        if 'wide' in k or 'igemm' in k or 'ars' in k:
            print(k, {c: round(sum(x)/len(x),1) for c,x in v.items()})
PY
